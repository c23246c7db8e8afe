#!/usr/bin/env python3
"""Count instructions per kernel in a hipcc --cuda-device-only -S listing (VALU mix, SGPR-operand VALU)."""
import collections
import re
import sys


def kernels(path):
    name, body = None, []
    for line in open(path):
        m = re.match(r'^(_Z\S+):', line)
        if m:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if 's_endpgm' in line:
            yield name, body
            name = None
            continue
        body.append(line)


for name, body in kernels(sys.argv[1]):
    if len(sys.argv) > 2 and not re.search(sys.argv[2], name):
        continue
    c = collections.Counter()
    sgpr_valu = 0
    for line in body:
        t = line.split(';')[0].strip().split(None, 1)
        if not t or t[0].startswith('.') or t[0].endswith(':'):
            continue
        c[t[0]] += 1
        if t[0].startswith('v_') and len(t) > 1 and re.search(r'\bs\d+\b|\bs\[', t[1].split(',', 1)[-1]):
            sgpr_valu += 1
    v = sum(n for k, n in c.items() if k.startswith('v_'))
    print(f"{name}: VALU {v} (with SGPR operand {sgpr_valu}) |",
          ', '.join(f'{k}:{n}' for k, n in c.most_common(10)))
