#!/usr/bin/env python3
"""Instruction mix of a kernel's innermost loop from a hipcc --save-temps .s file.

    python3 scripts/isa_loop_stats.py attention-hip-amdgcn-amd-amdhsa-gfx950.s attn_fwd_kernelILi64ELb0ELb1ELi3E

Prints VGPR / spill counts of every matching kernel and, for the first loop (``Inner Loop Header``
up to its back-branch), the VALU instruction count and the top instructions.  Used to check that
a kernel change removed per-iteration address arithmetic (VALU-bound attention loops).
"""
import re
import sys
from collections import Counter


def kernel_body(text, key):
    m = re.search(r"^(_Z\S*" + re.escape(key) + r"\S*):", text, re.M)
    if not m:
        raise SystemExit(f"kernel {key!r} not found")
    body = text[m.end():]
    return m.group(1), body[:body.index("s_endpgm")]


def loop_lines(body):
    lines = body.splitlines()
    a = next(i for i, l in enumerate(lines) if "Inner Loop Header" in l)
    b = next(i for i in range(a + 1, len(lines)) if re.match(r"\s*s_branch \.LBB", lines[i]))
    return lines[a:b + 1]


def main():
    path, key = sys.argv[1], sys.argv[2]
    text = open(path).read()
    name, body = kernel_body(text, key)
    meta = text[text.index("amdhsa.kernels"):]
    for blk in meta.split("  - .")[1:]:
        n = re.search(r"\.name:\s+(\S+)", blk)
        if n and n.group(1) == name:
            v = re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)
            s = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1)
            print(f"{key}: vgpr {v}, spills {s}")
    loop = loop_lines(body)
    ops = Counter(m.group(1) for l in loop if (m := re.match(r"\s*([sv]_\w+|ds_\w+|global_\w+|buffer_\w+)", l)))
    print(f"loop: {len(loop)} lines, VALU {sum(c for o, c in ops.items() if o.startswith('v_'))}")
    for o, c in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 16):
        print(f"  {c:4d} {o}")


if __name__ == "__main__":
    main()
