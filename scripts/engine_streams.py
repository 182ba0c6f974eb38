import sys, torch, json
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_engine_pipelined
m, sc = prepare_model(torch.device("cuda"), 20)
for st in (1, 2, 4, 8):
    print(json.dumps(measure_engine_pipelined(m, sc, 200, 20, streams=st)), flush=True)
