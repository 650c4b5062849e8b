"""Instruction histogram per kernel of a hipcc -S listing: python tools/isa_hist.py file.s [substr]"""
import collections, re, sys
s = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
parts = re.split(r'\n(?=_Z[A-Za-z0-9_]*:)', s)
for f in parts:
    m = re.match(r'(_Z[A-Za-z0-9_]*):', f)
    if not m or want not in m.group(1):
        continue
    body = f.split('.Lfunc_end')[0]
    c = collections.Counter(re.findall(r'^\s+([vsd][_a-z0-9]+|buffer_\w+|global_\w+)', body, re.M))
    print(m.group(1)[:70], sum(c.values()))
    print('   ', ' '.join('%s:%d' % kv for kv in c.most_common(40)))
