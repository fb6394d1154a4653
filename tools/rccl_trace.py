"""Kernel sequence of the last replayed training step of a rocprofv3
``--kernel-trace`` run, with the RCCL collectives marked (used for
``profiles/rccl_world1_graph_step_*.txt``).

    python tools/rccl_trace.py <kernel_trace.csv> [header lines...] > out.txt

The step is the span after the second-to-last ``adam_multi_kernel`` up to
and including the last one.  Queue ids (q1..) are the HIP hardware queues
the kernels were dispatched on (the capture's side streams show up as
separate queues).  On a one-rank communicator RCCL's all-reduce runs as
``oneRankReduce`` (a local copy-scale kernel): it exercises the capture of
the collective launch, not the ring / P2P transport of a multi-rank group.
"""
import csv
import re
import sys


def short(name):
    name = name.replace('(anonymous namespace)::', '')
    name = re.sub(r'\(.*', '', name)
    return name[:90]


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    adam = [i for i, r in enumerate(rows)
            if 'adam_multi_kernel' in r['Kernel_Name']]
    if len(adam) < 2:
        sys.exit('need at least two steps in the trace')
    step = rows[adam[-2] + 1:adam[-1] + 1]
    t0 = int(step[0]['Start_Timestamp'])
    t1 = max(int(r['End_Timestamp']) for r in step)
    is_rccl = [('rccl' in r['Kernel_Name'].lower() or
                'Reduce' in r['Kernel_Name'] or 'nccl' in r['Kernel_Name'])
               for r in step]
    total_rccl = sum(1 for r in rows if 'rccl' in r['Kernel_Name'].lower()
                     or 'oneRankReduce' in r['Kernel_Name'])
    for h in sys.argv[2:]:
        print(h)
    print('total RCCL dispatches in the run: {}'.format(total_rccl))
    print('step span {:.3f} ms, {} kernels, {} RCCL kernels inside it'.format(
        (t1 - t0) / 1e6, len(step), sum(is_rccl)))
    queues = {}
    for r, rc in zip(step, is_rccl):
        q = r.get('Queue_Id', r.get('Stream_Id', '0'))
        qn = queues.setdefault(q, 'q{}'.format(len(queues) + 1))
        s = int(r['Start_Timestamp']) - t0
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        tag = '  <== RCCL all_reduce (bucket)' if rc else ''
        name = ('rccl ' + short(r['Kernel_Name'])) if rc else \
            short(r['Kernel_Name'])
        print('{:9.1f} us {:8.1f} us  {:<4} {}{}'.format(
            s / 1e3, d / 1e3, qn, name, tag))


if __name__ == '__main__':
    main()
