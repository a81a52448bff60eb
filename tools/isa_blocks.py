"""Per-basic-block instruction classes of one kernel in a hipcc -S listing (blocks with > N instrs).
usage: python tools/isa_blocks.py <file.s> <mangled-name substring> [min-instructions] [top-k]"""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 100
top = int(sys.argv[4]) if len(sys.argv) > 4 else 10
s = open(path).read()
m = re.search(r'^(_Z\S*' + re.escape(pat) + r'\S*):', s, re.M)
i = m.start()
j = s.index('.Lfunc_end', i)
for b in re.split(r'\n(?=\.LBB)', s[i:j]):
    ins = re.findall(r'^\s+([vsdbg][a-z_0-9]+)', b, re.M)
    c = collections.Counter()
    for x in ins:
        if x.startswith('v_mfma'):
            c['mfma'] += 1
        elif x.startswith('v_'):
            c['valu'] += 1
        elif x.startswith('buffer_load'):
            c['vload'] += 1
        elif x.startswith('buffer_store'):
            c['vstore'] += 1
        elif x.startswith('ds_'):
            c['ds'] += 1
        elif x.startswith('s_'):
            c['salu'] += 1
        elif x.startswith('scratch'):
            c['scratch'] += 1
    if sum(c.values()) > mn:
        print(b.splitlines()[0][:60].strip(), dict(c))
        t = collections.Counter(x for x in ins if x.startswith('v_') and 'mfma' not in x)
        print('    ', t.most_common(top))
