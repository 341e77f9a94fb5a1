"""Static VALU count of one kernel by source function (DESIGN.md §4.4 per-phase table).

    hipcc -O3 -g --offload-arch=gfx950 --offload-device-only -S -o jd.s csrc/jd_kernels.hip ...
    python tools/isa_phases.py jd.s _ZN2jd12k_idct_colorILi1EEEvNS_8BatchDevE [--lines]

Each instruction is attributed to the source line of the `.loc` directive before it (the innermost
inlined frame), and each line of jd_kernels.hip to the function whose body contains it.  Counts
are static (every instruction once, whatever path or trip count runs it); the rare paths are
listed separately by function so that they can be left out of the common-path total.
"""
import collections
import re
import sys

SRC = "gpu-jpeg-decoder_amd/csrc/jd_kernels.hip"


def function_ranges(path):
    """[(first line, name)] of every function / lambda-hosting definition in the source."""
    defs = []
    pat = re.compile(r"^(?:template <[^>]*>\s*)?(?:__global__|__device__)[^(]*?\b(\w+)\s*\(")
    for i, line in enumerate(open(path), 1):
        m = pat.match(line)
        if m:
            defs.append((i, m.group(1)))
    return defs


def owner(defs, line):
    name = "?"
    for first, n in defs:
        if first > line:
            break
        name = n
    return name


def main():
    asm, sym = sys.argv[1], sys.argv[2]
    per_line = "--lines" in sys.argv
    defs = function_ranges(SRC)
    text = open(asm).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(sym + ":"))
    file_main = None
    for l in text:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', l)
        if m and m.group(2).endswith("jd_kernels.hip"):
            file_main = m.group(1)
            break
    cur = (None, 0)
    by_fn = collections.Counter()
    by_line = collections.Counter()
    total = 0
    for l in text[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            cur = (m.group(1), int(m.group(2)))
            continue
        if re.match(r"\s+v_", l):
            total += 1
            if cur[0] == file_main and cur[1] > 0:
                by_fn[owner(defs, cur[1])] += 1
                by_line[cur[1]] += 1
            else:
                by_fn["(header / line 0)"] += 1
    print(f"{sym}: {total} VALU (static)")
    for fn, n in by_fn.most_common():
        print(f"  {n:5d}  {fn}")
    if per_line:
        src = open(SRC).read().splitlines()
        for ln, n in sorted(by_line.items()):
            print(f"  {ln:5d} {n:4d}  {src[ln - 1].strip()[:100]}")


if __name__ == "__main__":
    main()
