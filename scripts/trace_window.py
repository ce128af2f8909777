"""Print the kernels between consecutive launches of a marker kernel in a
rocprofv3 kernel trace (per-sweep / per-iteration breakdowns).
usage: trace_window.py TRACE.csv MARKER IDX [IDX...]"""
import csv
import re
import sys


def short(n):
    n = n.replace('cgx::(anonymous namespace)::', '').replace('rocprim::ROCPRIM_400200_NS::detail::', '')
    if 'trampoline' in n:
        m = re.search(r'wrapped_(\w+)', n)
        return 'rp:' + (m.group(1) if m else n[:40])
    return n.split('(')[0].split('<')[0].replace('void ', '')[:40]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
seq = [(short(r['Kernel_Name']), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3,
        int(r['Start_Timestamp']), r['Grid_Size_X']) for r in rows]
idx = [i for i, s in enumerate(seq) if s[0] == sys.argv[2]]
print(len(idx), 'marker launches')
for k in map(int, sys.argv[3:]):
    a, b = idx[k], idx[k + 1]
    print('----', k, f'{(seq[b][2] - seq[a][2]) / 1e6:.3f} ms wall')
    tot = 0
    for s in seq[a:b]:
        tot += s[1]
        if s[1] > 20:
            print(f"{s[1]:9.1f} us {s[0]} grid={s[3]}")
    print(f'busy {tot / 1e3:.3f} ms')
