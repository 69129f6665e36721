"""Per-round kernel breakdown of a rocprofv3 kernel trace (dev tool): trace_rounds.py <dir> lo-hi [lo-hi...]"""
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rs = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
seq = [(r['Kernel_Name'].split('(')[0].replace('void ', '').replace('kb::', ''),
        (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, int(r['Start_Timestamp'])) for r in rs]
idx = [i for i, (n, _, _) in enumerate(seq) if n == 'k_log_mark']
for span in sys.argv[2:]:
    lo, hi = map(int, span.split('-'))
    agg = collections.defaultdict(float)
    wall = 0
    for rr in range(lo, hi):
        a, b = idx[rr], idx[rr + 1]
        wall += (seq[b][2] - seq[a][2]) / 1e3
        w = collections.Counter()
        for n, d, _ in seq[a:b]:
            if n in ('k_proc', 'k_route', 'k_kp_insert', 'k_sort_inbox'):
                agg[f'{n}_w{w[n]}'] += d; w[n] += 1
            else:
                agg[n] += d
    tot = sum(agg.values()) / (hi - lo)
    print(f'rounds {lo}-{hi}: kernel us/round {tot:.0f}, wall us/round {wall/(hi-lo):.0f}')
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:14]:
        print(f'   {k:28s} {v/(hi-lo):9.1f}')
