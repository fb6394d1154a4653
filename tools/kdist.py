"""Per-call duration distribution of kernels matching a pattern in a
rocprofv3 kernel_trace.csv:  python tools/kdist.py trace.csv pattern..."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:]
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    for p in pats:
        if p in n:
            grid = int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1)
            dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            d[n[:60]].append((dur, grid))
for k, v in d.items():
    c = collections.Counter((round(x[0] / 5) * 5, x[1]) for x in v)
    print(k, len(v))
    for (dur, grid), n in sorted(c.items(), key=lambda t: -t[1])[:8]:
        print('   %7.1f us  grid %6d  x%d' % (dur, grid, n))
