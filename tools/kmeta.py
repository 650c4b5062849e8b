"""Resource usage per kernel from a hipcc -S listing: python tools/kmeta.py file.s [substr]"""
import re, sys
s = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r'\n\s+- \.agpr_count', s)[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk)
    if not name or want not in name.group(1):
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', blk) or [None, '?'])[1]
    print('%-70s vgpr %s sgpr %s scratch %s lds %s' % (name.group(1)[:70], g('vgpr_count'), g('sgpr_count'),
          g('private_segment_fixed_size'), g('group_segment_fixed_size')))
