"""Per-step spans of a rocprofv3 kernel trace (split at the Adam kernel) and,
for the slowest step, the kernels that grew most vs the median step.

    python tools/step_outliers.py run_kernel_trace.csv [marker]
"""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'adam_multi'
    rows = sorted(csv.DictReader(open(path)),
                  key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    steps = [rows[a + 1:b + 1] for a, b in zip(ends, ends[1:])]
    spans = []
    for st in steps:
        t0 = int(st[0]['Start_Timestamp'])
        t1 = int(st[-1]['End_Timestamp'])
        busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp'])
                   for r in st)
        spans.append(((t1 - t0) / 1e6, busy / 1e6, len(st)))
    for i, (s, b, n) in enumerate(spans):
        print('step %2d span %.3f ms busy %.3f ms kernels %d' % (i, s, b, n))
    med = statistics.median(s for s, _, _ in spans)

    def agg(st):
        d = collections.defaultdict(float)
        for r in st:
            d[r['Kernel_Name'][:90]] += (int(r['End_Timestamp']) -
                                         int(r['Start_Timestamp'])) / 1e3
        return d
    slow = max(range(len(spans)), key=lambda i: spans[i][0])
    ref = min(range(len(spans)), key=lambda i: abs(spans[i][0] - med))
    a, b = agg(steps[slow]), agg(steps[ref])
    diff = sorted(((a[k] - b.get(k, 0.0), k) for k in a), reverse=True)[:12]
    print('slowest step %d vs median-like step %d:' % (slow, ref))
    for d, k in diff:
        print('  %+8.1f us  %s' % (d, k))


if __name__ == '__main__':
    main()
