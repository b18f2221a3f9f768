#!/usr/bin/env python3
"""VALU / LDS / VMEM instruction counts of one kernel's hot phase in an ISA
listing (make -C storage-engine_amd isa): per basic block and in total, for
checking an instruction-count change before a GPU run.
Usage: tools/isa_count.py <file.s> <kernel-symbol-substring> [first-barrier-index]"""
import re
import sys


def kernel_body(path, sub):
    s = open(path).read()
    m = re.search(r'^(_Z\S*' + re.escape(sub) + r'\S*):', s, re.M)
    if not m:
        sys.exit("no kernel matching %s" % sub)
    i = m.start()
    return m.group(1), s[i:s.index('.Lfunc_end', i)].split('\n')


def main():
    path, sub = sys.argv[1], sys.argv[2]
    name, body = kernel_body(path, sub)
    tot = {'v': 0, 'ds': 0, 'vm': 0, 's': 0}
    for l in body:
        t = l.strip()
        if not t or t.startswith((';', '.')) or t.endswith(':'):
            continue
        op = t.split()[0]
        k = 'v' if op.startswith('v_') else 'ds' if op.startswith('ds_') else \
            'vm' if op.startswith(('buffer_', 'global_')) else 's' if op.startswith('s_') else None
        if k:
            tot[k] += 1
    print(name[:140])
    print("static instruction counts (whole kernel):", tot)


if __name__ == "__main__":
    main()
