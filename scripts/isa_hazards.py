"""Software-managed hazards (manually inserted wait states) in libmsa.so's gfx950 code object.

hipcc's hazard recognizer pads the instructions it emits itself with `s_nop`; it inserts nothing in
front of or inside an inline-asm string, so hand-written asm must carry its own wait states.  A short
one reads a stale value on some waves of some launches -- wrong results that depend on issue timing.
Round 5's cflow_kernel had 47 DPPs reading their source one wait state after its VALU write.

For every consumer instruction of the classes below, this walks back over all control-flow predecessors
(fall-through and every branch that targets an address on the way) until the class's wait states have
been counted (one per instruction, N + 1 for an `s_nop N`) and reports each producer found inside them:

  dpp_vgpr     VALU writes a VGPR          -> a DPP op reads it (any VGPR operand, the `old`
                                              destination included, as LLVM's recognizer counts it)  2
  dpp_exec     VALU writes EXEC (v_cmpx)   -> a DPP op                                               5
  m0_lds       SALU writes M0              -> an LDS add-TID op, or a VMEM load into LDS              1
  sgpr_vmem    VALU writes an SGPR         -> a VMEM op reads that SGPR (address / resource)          5
  lane_select  VALU writes an SGPR         -> v_readlane / v_writelane selects its lane with it       4

Used by tests/test_host.py::test_asm_hazards_have_their_wait_states; run alone it prints the sites.

    python scripts/isa_hazards.py [path/to/libmsa.so]
"""
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import waitloops  # noqa: E402

VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
SREG = re.compile(r"\bs(\d+)\b|\bs\[(\d+):(\d+)\]|\b(vcc)\b|\b(m0)\b|\b(exec)\b")
TARGET = re.compile(r"<(.+?)(?:\+0x([0-9a-f]+))?>")
NO_FALLTHROUGH = ("s_branch", "s_endpgm", "s_setpc_b64", "s_trap")
VMEM = ("buffer_", "global_", "flat_", "scratch_")
DPP_CTRL = re.compile(r"\s(row_|wave_|quad_perm|bank_mask|bound_ctrl)")


def vregs(text: str):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def sregs(text: str):
    """SGPR names in an operand string: 's<k>' per register, 'vcc' (vcc_lo/hi as one), 'm0', 'exec'."""
    out = set()
    for m in SREG.finditer(text):
        if m.group(1) is not None:
            out.add(f"s{m.group(1)}")
        elif m.group(2) is not None:
            out.update(f"s{k}" for k in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add(m.group(4) or m.group(5) or m.group(6))
    return out


def operands(ops: str):
    """Operand strings of an instruction (DPP / memory modifiers stripped from the last one)."""
    head = DPP_CTRL.split(" " + ops, maxsplit=1)[0]
    return [o.strip() for o in head.split(",") if o.strip()]


def is_valu(mn: str) -> bool:
    return mn.startswith("v_")


def valu_vgpr_writes(mn, ops):
    if not is_valu(mn) or mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
        return set()
    o = operands(ops)
    return vregs(o[0].split()[0]) if o else set()


def valu_sgpr_writes(mn, ops):
    """SGPRs (incl. vcc, exec) a VALU instruction writes: its destination when scalar (v_readlane,
    v_readfirstlane, v_cmp*), or the carry-out / scale SGPR of a VOP3b op (second operand)."""
    if not is_valu(mn):
        return set()
    o = operands(ops)
    if not o:
        return set()
    out = sregs(o[0].split()[0]) if not vregs(o[0].split()[0]) else set()
    if mn.startswith("v_cmpx"):  # writes EXEC besides its printed destination
        out.add("exec")
    if len(o) > 1 and ("_co_" in mn or "div_scale" in mn):
        out |= sregs(o[1])
    return out


def salu_writes_m0(mn, ops):
    o = operands(ops)
    return mn.startswith("s_") and bool(o) and o[0] == "m0"


def wait_states(mn: str, ops: str) -> int:
    if mn == "s_nop":
        return int(ops.split()[0], 0) + 1
    return 1


def lds_m0_consumer(mn, ops):
    return "addtid" in mn or (mn.startswith(VMEM) and ("_lds" in mn or re.search(r"\blds\b", ops) is not None))


def consumers(mn, ops):
    """[(class, needed wait states, producer predicate)] this instruction is the consumer of."""
    out = []
    if mn.endswith("_dpp"):
        reads = vregs(" ".join(operands(ops)))
        out.append(("dpp_vgpr", 2, lambda m, o, r=reads: valu_vgpr_writes(m, o) & r))
        out.append(("dpp_exec", 5, lambda m, o: {"exec"} & valu_sgpr_writes(m, o)))
    if lds_m0_consumer(mn, ops):
        out.append(("m0_lds", 1, lambda m, o: {"m0"} if salu_writes_m0(m, o) else set()))
    if mn.startswith(VMEM):
        reads = sregs(" ".join(operands(ops))) - {"exec", "m0"}
        if reads:
            out.append(("sgpr_vmem", 5, lambda m, o, r=reads: valu_sgpr_writes(m, o) & r))
    if mn.startswith(("v_readlane", "v_writelane")):
        o = operands(ops)
        if len(o) >= 3:
            sel = sregs(o[2])
            if sel:
                out.append(("lane_select", 4, lambda m, oo, r=sel: valu_sgpr_writes(m, oo) & r))
    return out


def hazards(insts):
    """[(class, consumer_addr, consumer_text, producer_addr, producer_text, wait_states_between, regs)]"""
    base = waitloops.base_of(insts)
    index = {a: k for k, (a, _, _) in enumerate(insts)}
    preds = {k: [] for k in range(len(insts))}
    for k, (a, mn, ops) in enumerate(insts):
        if k + 1 < len(insts) and mn not in NO_FALLTHROUGH:
            preds[k + 1].append(k)
        if mn.startswith(("s_branch", "s_cbranch")):
            m = TARGET.search(ops)
            if m:
                tgt = base + int(m.group(2), 16) if m.group(2) else base
                if tgt in index:
                    preds[index[tgt]].append(k)
    bad = []
    for k, (a, mn, ops) in enumerate(insts):
        for cls, need, prod in consumers(mn, ops):
            seen = set()
            stack = [(p, 0) for p in preds[k]]
            while stack:
                j, ws = stack.pop()
                if (j, ws) in seen:
                    continue
                seen.add((j, ws))
                aj, mj, oj = insts[j]
                hit = prod(mj, oj)
                if hit:
                    bad.append((cls, a, f"{mn} {ops}".strip(), aj, f"{mj} {oj}".strip(), ws, sorted(hit)))
                    continue
                ws2 = ws + wait_states(mj, oj)
                if ws2 < need:
                    stack.extend((p, ws2) for p in preds[j])
    return bad


def dpp_hazards(insts):
    """The dpp_vgpr class alone, as (consumer_addr, consumer, producer_addr, producer, ws, vgpr)."""
    return [(a, t, aw, tw, ws, int(r[0][1:]) if isinstance(r[0], str) else r[0])
            for cls, a, t, aw, tw, ws, r in hazards(insts) if cls == "dpp_vgpr"]


def scan(so: Path, prefixes=None):
    """{function: (number of consumer instructions by class, [hazards])} for functions with consumers"""
    out = {}
    for name, insts in waitloops.functions(waitloops.disassemble(so)).items():
        if prefixes and not name.startswith(prefixes):
            continue
        counts = {}
        for _, mn, ops in insts:
            for cls, _, _ in consumers(mn, ops):
                counts[cls] = counts.get(cls, 0) + 1
        if counts:
            out[name] = (counts, hazards(insts))
    return out


if __name__ == "__main__":
    so = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parent.parent / \
        "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    total = 0
    for name, (counts, bad) in sorted(scan(so).items()):
        total += len(bad)
        if bad or "-v" in sys.argv:
            print(f"{len(bad):3d} short  {counts}  {name[:100]}")
        for cls, a, t, aw, tw, ws, r in bad[:4]:
            print(f"        [{cls}] {tw[:50]:50s} @{aw:#x} -> {ws} wait state(s) -> {t[:50]} @{a:#x} {r}")
    print(f"total short: {total}")
