"""Print the instruction schematic of a kernel's hottest loop from hipcc --save-temps assembly
(development tool): M = MFMA, R/W = LDS read/write (with width), G = global load, [..] = waits."""
import re
import sys


def main(path, kname):
    s = open(path).read().split('\n')
    a = [i for i, l in enumerate(s) if l.startswith(kname)][0]
    b = [i for i, l in enumerate(s) if i > a and l.startswith('.Lfunc_end')][0]
    lines = s[a:b]
    cur, cnt, start = 'entry', {'entry': 0}, {'entry': 0}
    for i, l in enumerate(lines):
        m = re.match(r'^(\.LBB\d+_\d+):', l)
        if m:
            cur = m.group(1)
            cnt[cur] = 0
            start[cur] = i
        elif 'v_mfma' in l:
            cnt[cur] += 1
    loop = max(cnt, key=cnt.get)
    out = []
    for l in lines[start[loop] + 1:]:
        l = l.strip()
        if l.startswith('.LBB'):
            break
        op = l.split(' ')[0] if l else ''
        if op.startswith('v_mfma'):
            out.append('M')
        elif op.startswith('ds_read') or op.startswith('ds_load'):
            out.append('R' + op.split('_')[-1])
        elif op.startswith('ds_write') or op.startswith('ds_store'):
            out.append('W' + op.split('_')[-1])
        elif op.startswith('global_load'):
            out.append('G')
        elif op.startswith('s_waitcnt'):
            out.append('[' + l[10:] + ']')
        elif op.startswith('s_barrier'):
            out.append('BAR')
    print(loop, 'mfma', cnt[loop])
    print(' '.join(out))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
