"""Per-step kernel timeline from a rocprofv3 ``kernel_trace.csv``.

Splits the dispatch stream at the optimizer kernel (one multi-tensor HIP Adam
launch per
training step), takes the LAST complete step and prints: wall span, summed
kernel time, kernel count, idle gaps and a per-kernel-name table.

    python tools/step_trace.py \
        gpurun_out/prof/.../run_kernel_trace.csv [marker]

(or the ``run_results.db`` rocprofv3 writes by default.)
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'adam_multi_kernel'
    if path.endswith('.db'):
        import sqlite3
        con = sqlite3.connect(path)
        rows = [{'Kernel_Name': n, 'Start_Timestamp': a, 'End_Timestamp': b}
                for n, a, b in con.execute(
                    'select name, start, end from kernels')]
    else:
        rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    if len(ends) < 2:
        print('marker %r found %d times' % (marker, len(ends)))
        return
    a, b = ends[-2] + 1, ends[-1] + 1
    step = rows[a:b]
    t0 = int(step[0]['Start_Timestamp'])
    t1 = int(step[-1]['End_Timestamp'])
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp'])
               for r in step)
    gaps = 0
    prev_end = t0
    for r in step:
        s = int(r['Start_Timestamp'])
        if s > prev_end:
            gaps += s - prev_end
        prev_end = max(prev_end, int(r['End_Timestamp']))
    print('step span %.3f ms, kernel time %.3f ms, idle %.3f ms, kernels %d'
          % ((t1 - t0) / 1e6, busy / 1e6, gaps / 1e6, len(step)))
    agg = collections.OrderedDict()
    for r in step:
        name = r['Kernel_Name']
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        n, t = agg.get(name, (0, 0))
        agg[name] = (n + 1, t + d)
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print('%7.3f ms %4d x %7.1f us  %s' % (t / 1e6, n, t / n / 1e3,
                                             name[:120]))
    if '--seq' in sys.argv:
        for r in step:
            d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            print('%8.1f us %7.1f  %s' % (
                (int(r['Start_Timestamp']) - t0) / 1e3, d / 1e3,
                r['Kernel_Name'][:100]))


if __name__ == '__main__':
    main()
