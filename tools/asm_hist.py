#!/usr/bin/env python3
"""Static VALU instruction histogram of the kernels in a hipcc -S listing
(`make -C ntt-gpu-qtesla_amd asm` -> build/ntt_kernels.s, build/nussbaumer.s).

    python tools/asm_hist.py build/ntt_kernels.s [substring ...]

Prints, per kernel whose mangled name contains every substring, the count of
each v_* opcode (the kernels' work loops are straight-line code, so the
static counts are the per-unit dynamic counts up to the loop control), and
returns them as a dict from `hist()` for tools/valu_summary.py.
"""
import collections
import re
import sys


def kernels(path):
    """{mangled name: [instruction lines]} of a hipcc -S listing."""
    out, cur = {}, None
    for line in open(path):
        m = re.match(r'^(_Z\w+):\s', line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if line.startswith('.Lfunc_end'):
                cur = None
                continue
            out[cur].append(line)
    return out


def hist(path, *subs):
    res = {}
    for name, lines in kernels(path).items():
        if all(s in name for s in subs):
            c = collections.Counter()
            for l in lines:
                m = re.match(r'\s+(v_\w+)', l)
                if m:
                    c[m.group(1)] += 1
            res[name] = c
    return res


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, c in hist(path, *subs).items():
        print(f"{name}: {sum(c.values())} VALU")
        for op, k in c.most_common():
            print(f"  {op:28s} {k}")


if __name__ == "__main__":
    main()
