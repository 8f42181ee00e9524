"""Per-basic-block instruction mix of one kernel in a gfx950 .s file.

usage: python bench/isa_blocks.py FILE.s SUBSTRING   (kernel symbol substring)
"""
import re
import sys


def main(path, sub):
    s = open(path).read()
    names = [l.split(':')[0] for l in s.splitlines() if l.startswith('_ZN') and sub in l.split(':')[0]]
    name = names[0]
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    blocks, cur = [], ['entry', []]
    for l in s[i:j].splitlines():
        if re.match(r'^\.LBB\d+_\d+:', l):
            blocks.append(cur)
            cur = [l.split(':')[0] + ' ' + (l.split(';', 1)[1].strip() if ';' in l else ''), []]
        elif l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'):
            cur[1].append(l.strip())
    blocks.append(cur)
    print(name)
    for nm, ins in blocks:
        v = sum(1 for x in ins if x.startswith('v_') and 'mfma' not in x)
        m = sum(1 for x in ins if 'mfma' in x)
        ds = sum(1 for x in ins if x.startswith('ds_'))
        gl = sum(1 for x in ins if x.startswith(('global_', 'buffer_')))
        sa = sum(1 for x in ins if x.startswith('s_'))
        print(f"{nm[:64]:64s} n={len(ins):4d} valu={v:4d} mfma={m:2d} ds={ds:3d} glob={gl:3d} salu={sa:3d}")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
