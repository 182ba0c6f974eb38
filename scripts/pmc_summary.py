"""Summarize rocprofv3 PMC runs (set*/pmc_counter_collection.csv) per (kernel, grid) dispatch class."""
import csv, collections, glob, sys
d = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f'{d}/set*/pmc_counter_collection.csv')):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f)):
        k = (r['Dispatch_Id'])
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        meta[k] = (r['Kernel_Name'][:64], r['Grid_Size'], int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    for k, v in acc.items():
        name, grid, dur = meta[k]
        if 'conv' not in name and 'wgrad' not in name: continue
        for c, x in v.items(): per[(name, grid)][c].append(x)
        per[(name, grid)]['dur_us'].append(dur / 1e3)
for (name, grid), v in per.items():
    m = {c: sum(x) / len(x) for c, x in v.items()}
    print(f'== {name} grid={grid}  dur={m["dur_us"]:.1f}us')
    wc = m.get('SQ_WAVE_CYCLES', 1)
    for c in sorted(m):
        extra = ''
        if c.startswith('SQ_WAIT') or c.startswith('SQ_ACTIVE'):
            extra = f'  ({100 * m[c] / wc:.1f}% of wave cycles)'
        print(f'   {c:36s} {m[c]:.4g}{extra}')
    if 'SQ_INSTS_MFMA' in m:
        mf = m['SQ_INSTS_MFMA']
        print(f'   per MFMA: VALU {m.get("SQ_INSTS_VALU",0)/mf:.2f} SALU {m.get("SQ_INSTS_SALU",0)/mf:.2f} LDS {m.get("SQ_INSTS_LDS",0)/mf:.2f} VMEM {m.get("SQ_INSTS_VMEM",0)/mf:.2f}')
    if 'TCC_HIT_sum' in m:
        print(f'   L2 hit rate {100*m["TCC_HIT_sum"]/(m["TCC_HIT_sum"]+m["TCC_MISS_sum"]):.1f}%')
