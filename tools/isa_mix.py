"""Instruction mix of the kernels in a hipcc `-S` listing (gfx950).

usage: python tools/isa_mix.py <file.s> <substring of the mangled kernel name> [top-N]
Prints, per matching kernel, the static instruction count by mnemonic and the register metadata
(.vgpr_count / .agpr_count / .sgpr_count / LDS) from the code-object notes.
"""
import re
import sys
from collections import Counter


def kernels(text):
    starts = [(m.start(), m.group(1)) for m in re.finditer(r'^(_Z\S+):\s*(?:;.*)?$', text, re.M)]
    for i, (pos, name) in enumerate(starts):
        end = starts[i + 1][0] if i + 1 < len(starts) else len(text)
        yield name, text[pos:end]


def meta(text, name):
    m = re.search(r'\.name:\s+' + re.escape(name) + r'\n(.*?)(?:\n\s+- \.|\Z)', text, re.S)
    out = {}
    blk = text[max(0, text.find('.name:           ' + name) - 4000):text.find('.name:           ' + name) + 2000]
    for key in ('.vgpr_count', '.agpr_count', '.sgpr_count', '.group_segment_fixed_size', '.vgpr_spill_count'):
        mm = re.findall(re.escape(key) + r':\s+(\d+)', blk)
        if mm:
            out[key] = mm[-1]
    return out


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    text = open(path).read()
    for name, body in kernels(text):
        if pat not in name:
            continue
        ins = re.findall(r'^\s+([vsdgb][a-z_0-9]+)\b', body, re.M)
        ins = [i for i in ins if re.match(r'(v_|s_|ds_|buffer_|global_)', i)]
        c = Counter(ins)
        cls = Counter()
        for k, v in c.items():
            cls['mfma' if 'mfma' in k else k.split('_')[0]] += v
        print(f'{name}: {len(ins)} instructions  {dict(cls)}  {meta(text, name)}')
        for k, v in c.most_common(top):
            print(f'  {k:32s} {v}')


if __name__ == '__main__':
    main()
