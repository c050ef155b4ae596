"""Opcode-class histogram of one kernel's loops, from the gfx950 assembly
(make -C firedancer_amd/csrc asm).  Finds the loops by their back edges
(a branch to an earlier label), prints each loop's size and instruction
classes, and -- with --weights 'LINE:TRIPS,...' -- a trip-weighted total per
class for the loops named by their first line.

    python tools/isa_hist.py firedancer_amd/csrc/fdgpu_kernels.s \
        --kernel _ZN12_GLOBAL__N_122fdgpu_verify_hs_kernelILb0E [--weights 12345:33]
"""
import argparse
import collections
import json
import re


def klass(op):
    if op.startswith("v_mad_u64_u32"):
        return "v_mad_u64_u32"
    if op.startswith(("v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64", "v_add_co_u32", "v_addc_co_u32",
                      "v_sub_co_u32", "v_subb_co_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24",
                      "v_mul_u32_u24", "v_alignbit_b32", "v_bfi_b32", "v_cndmask_b32", "v_bitop3_b32")):
        return op.split("_e32")[0].split("_e64")[0].split("_dpp")[0]
    if op.startswith(("v_mov_b32", "v_mov_b64", "v_accvgpr", "v_readlane", "v_writelane", "v_readfirstlane")):
        return "v_mov/lane"
    if op.startswith(("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_add3_u32", "v_lshl_add_u32", "v_add_lshl_u32")):
        return "v_add/sub_u32"
    if op.startswith(("v_and_b32", "v_or_b32", "v_xor_b32", "v_and_or_b32", "v_or3_b32", "v_xor3_b32",
                      "v_not_b32", "v_lshrrev_b32", "v_lshlrev_b32", "v_ashrrev_i32", "v_bfe_u32", "v_lshl_or_b32",
                      "v_perm_b32")):
        return "v_logic/shift32"
    if op.startswith("v_cmp"):
        return "v_cmp"
    if op.startswith("v_"):
        return "v_other"
    if op.startswith(("scratch_", "buffer_")):
        return "scratch/buffer"
    if op.startswith("global_load_lds"):
        return "global_load_lds"
    if op.startswith("global_"):
        return "global"
    if op.startswith("ds_"):
        return "ds (LDS)"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_"):
        return "salu/branch"
    return "other"


def parse(path, kernel):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel) and l.rstrip().endswith(
        tuple([":", l.split(":")[0] + ":"])) or (l.startswith(kernel) and ":" in l.split(";")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    body = []                                        # (lineno, kind, text)
    for i in range(start + 1, end + 1):
        t = lines[i].split(";")[0].strip()
        if not t or t.startswith("."):
            if re.match(r"^\.LBB\w+:", lines[i].strip()):
                body.append((i + 1, "label", t.rstrip(":")))
            continue
        if re.match(r"^\.LBB\w+:", t):
            body.append((i + 1, "label", t.rstrip(":")))
            continue
        body.append((i + 1, "insn", t))
    return body


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--weights", default="",
                    help="LINE:TRIPS or FIRST-LAST:TRIPS,... for the loops starting at LINE (spanning FIRST-LAST)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    body = parse(args.asm, args.kernel)
    label_pos = {t: k for k, (ln, kind, t) in enumerate(body) if kind == "label"}
    loops = []
    for k, (ln, kind, t) in enumerate(body):
        if kind != "insn" or not t.startswith("s_cbranch") and not t.startswith("s_branch"):
            continue
        tgt = t.split()[-1]
        if tgt in label_pos and label_pos[tgt] < k:
            loops.append((label_pos[tgt], k))
    total = collections.Counter(klass(t.split()[0]) for _, kind, t in body if kind == "insn")
    print(f"kernel {args.kernel}: {sum(total.values())} instructions (static)")
    weights = {}
    for w in (w for w in args.weights.split(",") if w):
        key, trips = w.split(":")
        weights[tuple(int(x) for x in key.split("-")) if "-" in key else int(key)] = float(trips)
    weighted = collections.Counter()
    report = {"static_total": dict(total), "loops": []}
    for a, b in loops:
        ins = [t for _, kind, t in body[a:b + 1] if kind == "insn"]
        h = collections.Counter(klass(t.split()[0]) for t in ins)
        first = body[a][0]
        nested = sum(1 for c, d in loops if a < c and d < b)
        print(f"loop lines {first}-{body[b][0]}: {len(ins)} insns, {nested} inner loops; "
              + ", ".join(f"{k} {v}" for k, v in h.most_common(8)))
        report["loops"].append({"first_line": first, "last_line": body[b][0], "insns": len(ins),
                                "inner_loops": nested, "classes": dict(h)})
        wt = weights.get((first, body[b][0]), weights.get(first))
        if wt:
            for k, v in h.items():
                weighted[k] += v * wt
    if weighted:
        tot = sum(weighted.values())
        print(f"trip-weighted total over the named loops: {tot:.0f} instructions per lane")
        for k, v in weighted.most_common():
            print(f"  {k:22s} {v:10.0f}  {100 * v / tot:5.1f}%")
        report["weighted"] = {k: v for k, v in weighted.items()}
    if args.json:
        json.dump(report, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
