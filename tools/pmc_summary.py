"""Per-(kernel, grid) averages of a rocprofv3 ``--pmc`` run's
``counter_collection.csv`` (one line per kernel and grid size).

    python tools/pmc_summary.py <counter_collection.csv> [filter] > out

(filter: a kernel-name substring, e.g. ``dgmc::``.)
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name']
        if filt not in name:
            continue
        base = name.replace('(anonymous namespace)::', '')
        key = (base.split('(')[0], r['Grid_Size'])
        sums[key][r['Counter_Name']] += float(r['Counter_Value'])
        disp[key].add(r['Dispatch_Id'])
    for key in sorted(sums):
        n = max(1, len(disp[key]))
        vals = ' '.join('%s=%d' % (c, v / n)
                        for c, v in sorted(sums[key].items()))
        print('%s grid=%s %s' % (key[0], key[1], vals))


if __name__ == '__main__':
    main()
