"""Static VGPR-spill report of one kernel in a hipcc -S listing (diagnostic).

Usage: python tools/spills.py build/rtw_render.s KERNEL_SUBSTRING
Prints the kernel's scratch loads/stores grouped by the innermost loop header
they sit in, with the source line of that header (build with -gline-tables-only
for the line numbers).
"""
import collections
import re
import sys


def main(path, key):
    s = open(path).read().split('\n')
    starts = [i for i, l in enumerate(s) if re.match(r'^_Z\S*:', l) and key in l]
    if not starts:
        sys.exit(f'no kernel matching {key}')
    st = starts[0]
    en = next(i for i in range(st, len(s)) if s[i].strip().startswith('.Lfunc_end'))
    hdr_line = {}
    cur_loc = 0
    for i in range(st, en):
        m = re.search(r'\.loc\s+0\s+(\d+)', s[i])
        if m and int(m.group(1)):
            cur_loc = int(m.group(1))
        m = re.match(r'^\.L(BB\S+):.*Loop Header', s[i])
        if m:
            nxt = next((re.search(r'\.loc\s+0\s+(\d+)', s[j]) for j in range(i, min(i + 60, en))
                        if re.search(r'\.loc\s+0\s+([1-9]\d*)', s[j])), None)
            hdr_line[m.group(1)] = int(nxt.group(1)) if nxt else cur_loc
    cnt = collections.Counter()
    hdr, depth = '-', 0
    for i in range(st, en):
        m = re.search(r'Header=(BB\S+) Depth=(\d+)', s[i]) or re.search(r'^\.L(BB\S+):.*Loop Header: Depth=(\d+)', s[i])
        if m:
            hdr, depth = m.group(1), int(m.group(2))
        elif re.match(r'^\.LBB\S+:\s*$', s[i]) or re.match(r'^\.LBB\S+:\s*;\s*%bb', s[i]):
            if 'Loop' not in s[i]:
                hdr, depth = '-', 0
        if 'scratch_' in s[i]:
            cnt[(depth, hdr, 'store' if 'store' in s[i] else 'load')] += 1
    tot = sum(cnt.values())
    print(f'{s[st].rstrip(":")}: {tot} scratch ops')
    for (d, h, k), v in sorted(cnt.items(), key=lambda kv: (-kv[0][0], kv[0][1])):
        print(f'  depth {d} loop {h} (line {hdr_line.get(h, "?")}): {v} {k}')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
