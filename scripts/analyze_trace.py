"""Map one training step's conv kernel dispatches (rocprofv3 kernel trace) to U-Net layers; print TF/s."""
import csv, sys
sys.path.insert(0, '.')
from robotic_discovery_platform_amd.models.unet import unet_conv_specs

path = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32
size = 256
rows = [r for r in csv.DictReader(open(path))]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
specs = unet_conv_specs(4, 64, 3, True)
# spatial size per spec in forward order
D = 4; sizes = []
lv = [0, 0] + sum([[i, i] for i in range(1, D + 1)], []) + sum([[D - i, D - i] for i in range(1, D + 1)], [])
MAIN = ('conv_first_kernel', 'wgrad_first_bn_kernel', 'conv_igemm_kernel', 'conv_pp_kernel', 'conv_halo_kernel', 'conv_ring_kernel', 'conv_wgrad_kernel', 'conv_wgrad_halo_kernel', 'conv_wgrad_ring_kernel')
REDUCE = ('conv_splitk_reduce_kernel', 'wgrad_reduce_kernel')
conv = []  # main conv dispatches; a following split-K / slab reduce is folded into its time
for r in rows:
    name = r['Kernel_Name']
    if any(m in name for m in MAIN):
        r = dict(r)
        conv.append(r)
    elif conv and any(m in name for m in REDUCE):
        conv[-1]['End_Timestamp'] = r['End_Timestamp']
per_step = 18 + 17 + 18  # fwd + dgrad + wgrad
step = conv[-per_step:]
fwd, bwd = step[:18], step[18:]
def flops(sp, l):
    hw = (size >> l) ** 2
    cin = 27 if sp.packed else sp.cin
    return 2.0 * batch * hw * cin * 9 * sp.cout / (9 if sp.packed else 1) * (1 if not sp.packed else 1)
tot_t = 0; tot_f = 0
print(f"{'layer':42s} {'kind':6s} {'us':>8s} {'TF/s':>7s} grid")
for i, (sp, r) in enumerate(zip(specs, fwd)):
    f = 2.0 * batch * (size >> lv[i]) ** 2 * (27 if sp.packed else 9 * sp.cin) * sp.cout
    t = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot_t += t; tot_f += f
    print(f"{sp.name:42s} fwd    {t:8.1f} {f / t / 1e6:7.1f} {r['Grid_Size_X']}")
# backward order: per layer wgrad then dgrad (no dgrad for first)
order = []
for i in range(D, 0, -1):
    order += [9 + 2 * i - 1 + 1 - 1 + 0]  # placeholder
bo = []
idx = {sp.name: i for i, sp in enumerate(specs)}
names = []
for i in range(D, 0, -1):
    names += [f"up{i}.conv.double_conv.3", f"up{i}.conv.double_conv.0"]
for i in range(D, 0, -1):
    names += [f"down{i}.maxpool_conv.1.double_conv.3", f"down{i}.maxpool_conv.1.double_conv.0"]
names += ["inc.double_conv.3", "inc.double_conv.0"]
k = 0
for n in names:
    i = idx[n]; sp = specs[i]
    f = 2.0 * batch * (size >> lv[i]) ** 2 * (27 if sp.packed else 9 * sp.cin) * sp.cout
    for kind in (["wgrad", "dgrad"] if not sp.packed else ["wgrad"]):
        r = bwd[k]; k += 1
        t = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        tot_t += t; tot_f += f
        assert (kind == 'wgrad') == ('wgrad' in r['Kernel_Name']), (kind, r['Kernel_Name'])
        print(f"{n:42s} {kind:6s} {t:8.1f} {f / t / 1e6:7.1f} {r['Grid_Size_X']}")
print(f"conv total {tot_t/1e3:.2f} ms  {tot_f/tot_t/1e6:.1f} TF/s  (times include split-K / slab reduce kernels)")
