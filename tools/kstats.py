"""Summarise a rocprofv3 kernel_stats.csv: per-step ms by kernel."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
calls = sum(int(r['Calls']) for r in rows)
print('GPU busy per step: %.3f ms, kernels per step: %.0f'
      % (tot / 1e6 / steps, calls / steps))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print('%7.3f ms/step %6.1f calls/step %7.1f us  %s' % (
        float(r['TotalDurationNs']) / 1e6 / steps, int(r['Calls']) / steps,
        float(r['AverageNs']) / 1e3, r['Name'][:110]))
