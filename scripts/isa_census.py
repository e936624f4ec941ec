#!/usr/bin/env python3
"""Static per-loop instruction census of a kernel in the device assembly (`make -C hello-raytracing_amd asm`).

Splits one kernel's code into basic blocks, rebuilds the loop nest from the compiler's loop annotations
("Loop Header: Depth=N", "in Loop: Header=BBx Depth=N") and counts every block's instructions by class:
FP32 math (fma / mul / add / min / max / med3 / fma_mix / packed), transcendental (rcp, sqrt, rsq, ...),
compare, v_cndmask, move (v_mov / v_pk_mov), integer / address arithmetic, conversion, cross-lane
(readlane / readfirstlane / bpermute / mbcnt), LDS, vector memory, SALU, branches and waits.

Usage:
  python scripts/isa_census.py build/rt_kernels.s 'k_trace_splitILb1ELb0E' [--blocks]
  python scripts/isa_census.py build/rt_kernels.s 'k_trace_split_trisILi2ELi1ELi3ELb0E' --json out.json

Counts are static (one per instruction in the block), so a loop's total is the cost of one trip through
every block of its body (both arms of an if/else: SIMT runs both when the lanes disagree). The census names
each loop by what it touches (LDS node reads, buffer loads of spheres / triangles, ...) so the walk, leaf
and shading loops can be told apart; `--blocks` prints every block with its class counts.
"""
from __future__ import annotations

import argparse
import json
import re
import sys
from collections import Counter, OrderedDict

CLASSES = ["fp32", "trans", "cmp", "cndmask", "mov", "int", "cvt", "xlane", "valu_other",
           "lds", "vmem", "smem", "salu", "branch", "wait"]

TRANS = re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos|rcp_iflag)_")
FP32 = re.compile(r"^v_(pk_)?(fma|fmac|fmaak|fmamk|mul|add|sub|subrev|min|max|min3|max3|med3|mac|"
                  r"fma_mix|mad|ldexp|div_scale|div_fmas|div_fixup|frexp|fract|floor|ceil|trunc|rndne|"
                  r"minimum3|maximum3)_f(32|16)|^v_(fma_mix|fma_mixlo|fma_mixhi)_f(32|16)|^v_pk_(fma|mul|add)_f32")
CMP = re.compile(r"^v_cmpx?_")
CND = re.compile(r"^v_cndmask_")
MOV = re.compile(r"^v_(mov|pk_mov|mov_b64)_")
CVT = re.compile(r"^v_cvt_")
XLANE = re.compile(r"^(v_readlane|v_readfirstlane|v_writelane|v_mbcnt|ds_bpermute|ds_permute|ds_swizzle|v_permlane)")
INT = re.compile(r"^v_(add|sub|subrev|addc|subb|mul_lo|mul_hi|mad_u32|mad_i32|mad_u64|lshl|lshr|ashr|and|or|xor|"
                 r"not|bfe|bfi|bfm|ffbl|ffbh|bcnt|alignbit|alignbyte|min_u32|max_u32|min_i32|max_i32|"
                 r"lshl_add|add_lshl|lshl_or|and_or|or3|xad|add3|mul_u32|mul_i32|perm|cmp_class|sad|"
                 r"lshlrev|lshrrev|ashrrev|mad_u32_u24|mad_i32_i24|mul_u32_u24|med3_u32|med3_i32|bitop)")
LDS = re.compile(r"^ds_")
VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
SMEM = re.compile(r"^s_(load|buffer_load|store|dcache|memtime|memrealtime)")
BRANCH = re.compile(r"^s_(cbranch|branch|setpc|swappc|endpgm)")
WAIT = re.compile(r"^s_(waitcnt|nop|sleep|barrier|sethalt)")


def classify(op: str) -> str:
    if BRANCH.match(op):
        return "branch"
    if WAIT.match(op):
        return "wait"
    if SMEM.match(op):
        return "smem"
    if XLANE.match(op):
        return "xlane"
    if LDS.match(op):
        return "lds"
    if VMEM.match(op):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    if TRANS.match(op):
        return "trans"
    if CMP.match(op):
        return "cmp"
    if CND.match(op):
        return "cndmask"
    if MOV.match(op):
        return "mov"
    if CVT.match(op):
        return "cvt"
    if FP32.match(op):
        return "fp32"
    if INT.match(op):
        return "int"
    if op.startswith("v_"):
        return "valu_other"
    return "other"


LABEL = re.compile(r"^(\.LBB\d+_\d+):")
BBCOMMENT = re.compile(r"^; %bb\.(\d+):")
HDR = re.compile(r"Loop Header: Depth=(\d+)")
INLOOP = re.compile(r"in Loop: Header=(BB\d+_\d+) Depth=(\d+)")
PARENT = re.compile(r"Parent Loop (BB\d+_\d+) Depth=(\d+)")


def kernel_lines(path: str, key: str) -> list[str]:
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and key in l and not l.startswith("\t"):
            start = i
            break
    if start is None:
        sys.exit(f"no kernel matching {key!r}")
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end") or l.strip().startswith("s_endpgm"):
            out.append(l)
            break
        out.append(l)
    return out


def parse(lines: list[str]):
    blocks: "OrderedDict[str, dict]" = OrderedDict()
    cur = {"name": "entry", "loop": None, "depth": 0, "header": False, "ops": []}
    blocks["entry"] = cur
    parents: dict[str, str | None] = {}
    pending_parent: list[tuple[str, int]] = []
    for l in lines:
        s = l.strip()
        m = LABEL.match(l) or BBCOMMENT.match(l)
        if m:
            name = m.group(1) if LABEL.match(l) else f"%bb.{m.group(1)}"
            name = name.lstrip(".L")
            cur = {"name": name, "loop": None, "depth": 0, "header": False, "ops": []}
            blocks[name] = cur
            pending_parent = []
        if ";" in l:
            c = l[l.index(";"):]
            h = HDR.search(c)
            if h:
                cur["header"] = True
                cur["loop"] = cur["name"]
                cur["depth"] = int(h.group(1))
                # the innermost Parent Loop seen on the label lines is this header's parent
                parents[cur["name"]] = pending_parent[-1][0] if pending_parent else None
            ip = INLOOP.search(c)
            if ip and not cur["header"]:
                cur["loop"] = ip.group(1)
                cur["depth"] = int(ip.group(2))
            pp = PARENT.search(c)
            if pp:
                pending_parent.append((pp.group(1), int(pp.group(2))))
        if not s or s.startswith(";") or s.startswith(".") or LABEL.match(l):
            continue
        op = s.split()[0]
        cur["ops"].append(op)
    for b in blocks.values():
        if b["loop"] and b["loop"] not in parents:
            parents[b["loop"]] = None
    return blocks, parents


def tags(ops: list[str]) -> list[str]:
    t = []
    if any(o.startswith("ds_read_b128") for o in ops):
        t.append("lds-b128")
    if any(o.startswith("ds_read_b96") for o in ops):
        t.append("lds-b96")
    if any(o.startswith("v_fma_mix") for o in ops):
        t.append("fp16-slab")
    if any(o.startswith("buffer_load_dwordx4") for o in ops):
        t.append("buf-x4")
    if any(o.startswith("buffer_load_dwordx3") for o in ops):
        t.append("buf-x3")
    if any(o.startswith("v_sqrt") for o in ops):
        t.append("sqrt")
    if any(o.startswith("v_rcp") for o in ops):
        t.append("rcp")
    if any(o.startswith("global_store") or o.startswith("buffer_store") for o in ops):
        t.append("store")
    if any(o.startswith("v_ffbl") for o in ops):
        t.append("ctz")
    return t


def census(blocks, parents):
    loops: "OrderedDict[str, dict]" = OrderedDict()
    loops["(outside loops)"] = {"depth": 0, "parent": None, "self": Counter(), "blocks": 0, "tags": set()}
    for b in blocks.values():
        key = b["loop"] or "(outside loops)"
        if key not in loops:
            loops[key] = {"depth": b["depth"], "parent": parents.get(key), "self": Counter(), "blocks": 0,
                          "tags": set()}
        L = loops[key]
        L["blocks"] += 1
        L["tags"].update(tags(b["ops"]))
        for o in b["ops"]:
            L["self"][classify(o)] += 1
    # inclusive counts: a loop's own blocks plus its child loops'
    for k, L in loops.items():
        L["incl"] = Counter(L["self"])
    for k, L in sorted(loops.items(), key=lambda kv: -kv[1]["depth"]):
        p = L["parent"]
        if p and p in loops:
            loops[p]["incl"].update(L["incl"])
    return loops


def valu(c: Counter) -> int:
    return sum(c[k] for k in ("fp32", "trans", "cmp", "cndmask", "mov", "int", "cvt", "valu_other")) + c["xlane"]


def fmt_row(name, depth, c: Counter, extra=""):
    v = valu(c)
    fp = c["fp32"] + c["trans"]
    cols = " ".join(f"{c[k]:>5}" for k in CLASSES)
    share = f"{100.0 * fp / v:5.1f}" if v else "   - "
    return f"{'  ' * depth}{name:<{24 - 2 * depth}} {v:>5} {share} {cols} {extra}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--blocks", action="store_true", help="print every block")
    ap.add_argument("--json", help="write the census as JSON")
    a = ap.parse_args()
    blocks, parents = parse(kernel_lines(a.asm, a.kernel))
    loops = census(blocks, parents)
    hdr = f"{'loop (exclusive)':<24} {'VALU':>5} {'%FP':>5} " + " ".join(f"{k[:5]:>5}" for k in CLASSES)
    print(hdr)
    for k, L in loops.items():
        print(fmt_row(k, L["depth"], L["self"], ",".join(sorted(L["tags"]))))
    total = Counter()
    for b in blocks.values():
        for o in b["ops"]:
            total[classify(o)] += 1
    print(fmt_row("TOTAL (static)", 0, total))
    if a.blocks:
        print()
        for b in blocks.values():
            c = Counter(classify(o) for o in b["ops"])
            print(fmt_row(b["name"], b["depth"], c, f"[{b['loop']}] " + ",".join(tags(b["ops"]))))
    if a.json:
        out = {k: {"depth": L["depth"], "parent": L["parent"], "tags": sorted(L["tags"]),
                   "exclusive": dict(L["self"]), "inclusive": dict(L["incl"]),
                   "valu_exclusive": valu(L["self"]), "valu_inclusive": valu(L["incl"])}
               for k, L in loops.items()}
        json.dump({"kernel": a.kernel, "loops": out, "total": dict(total)}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
