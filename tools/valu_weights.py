"""Static-mix VALU issue weights per kernel (bench.py's busy_frac priced every
VALU instruction at 4 cycles).

    hipcc -O3 --offload-arch=gfx950 --offload-device-only -S -o jd.s csrc/jd_kernels.hip ...
    python tools/valu_weights.py jd.s profiles/valurate.txt profiles/r05_valu_weights.json

Each VALU instruction of a kernel is priced at the wave64 issue cycles tools/micro/valurate.hip
measured for its opcode and encoding (profiles/r04c_valurate.txt: ~2.6-2.8 cycles for v_add_u32,
v_sub_u32, v_and_b32, v_ashrrev_i32, v_mov_b32, v_add_f32, v_mul_f32 in the e32 encoding; ~3.5-3.8
for v_bitop3, v_fma_f32 and the e64 encoding of the full-rate ones; ~4.4-4.9 for shifts left, v_bfe,
24-bit and 32-bit multiplies, v_perm, v_med3, v_dot2, packed 16-bit ops; unmeasured opcodes 4.6).
The weight is the static mean over the kernel's instructions (each instruction once, whatever path
or trip count runs it), so it describes the mix, not the dynamic count.
"""
import json
import re
import sys

DEFAULT = 4.6


def rates(path):
    out = {}
    for line in open(path):
        m = re.match(r"(v_\w+)\s.*?([\d.]+) cyc", line)
        if m:
            out.setdefault(m.group(1), float(m.group(2)))
    # the e32 v_cndmask_b32 row of the table timed a chain through vcc (20 cycles): the e64 form's
    # 4.7 cycles is the instruction's own issue cost
    if "v_cndmask_b32_e64" in out:
        out["v_cndmask_b32"] = out["v_cndmask_b32_e64"]
    return out


def main():
    asm, table, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    rt = rates(table)
    e64_full = rt.get("v_add_u32_e64", 3.77)
    text = open(asm).read().splitlines()
    res = {}
    cur, ops = None, []
    for line in text:
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur, ops = m.group(1), []
            continue
        if cur and line.startswith(".Lfunc_end"):
            tot = n = full = 0
            for op in ops:
                base = re.sub(r"_(e32|e64|dpp|sdwa)$", "", op)
                if op.endswith("_e64") and rt.get(base, DEFAULT) < 3.0:
                    c = e64_full
                else:
                    c = rt.get(base, rt.get(op, DEFAULT))
                tot += c
                n += 1
                full += c < 3.0
            if n:
                name = re.sub(r"^_ZN2jd\d+", "", cur)
                res[cur] = {"name": name, "valu_static": n, "cycles_per_valu": round(tot / n, 3),
                            "full_rate_frac": round(full / n, 3)}
            cur = None
            continue
        if cur:
            t = line.strip().split()
            if t and t[0].startswith("v_") and not t[0].startswith(("v_mfma", "v_readlane", "v_readfirstlane", "v_writelane")):
                ops.append(t[0])
    json.dump({"source": "static ISA mix x profiles/r04c_valurate.txt", "kernels": res}, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(f"{v['name'][:40]:40s} {v['valu_static']:6d} {v['cycles_per_valu']:.3f} {v['full_rate_frac']:.3f}")


if __name__ == "__main__":
    main()
