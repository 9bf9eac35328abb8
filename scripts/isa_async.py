"""Asynchronous results used before their s_waitcnt in libmsa.so's gfx950 code object.

A DS (LDS) or VMEM load writes its destination VGPRs when it returns, not when it issues; the hardware
does not interlock on them, so every read -- or overwrite -- of such a VGPR must come after an
`s_waitcnt` that covers the load.  hipcc counts the loads it emits.  It does not count the loads of
inline asm (the flow / band / cflow kernels issue their ring and counter reads that way, with explicit
`s_waitcnt lgkmcnt(N)` asm and the outputs tied to the wait), and nothing stops it from copying, moving
or spilling an asm load's output register between the asm and the wait -- which reads a value that has
not landed yet (wrong results that depend on timing), or lets the late return overwrite a register
the compiler had reused.

Dataflow over every function's control-flow graph: the state is the ordered list of outstanding loads
(their destination registers) per counter.
  lgkmcnt: DS ops return in order among themselves; SMEM returns out of order.  After
           `s_waitcnt lgkmcnt(N)` the N most recent DS ops may still be outstanding (the SMEM ops may have
           been the ones that completed); SMEM entries clear only at lgkmcnt(0).
  vmcnt:   VMEM ops return in order; after `vmcnt(N)` the N most recent remain.
At a join the lists are merged aligned on their most recent entry (union per position).  Every
instruction's register operands are checked against the outstanding destinations (a later load writing
the same registers in order is not a conflict).  Calls and returns count as full waits (a callee's
prologue waits for everything).

Used by tests/test_host.py::test_async_loads_are_waited_for; run alone it prints the sites.

    python scripts/isa_async.py [path/to/libmsa.so]
"""
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import isa_hazards as H  # noqa: E402
import waitloops  # noqa: E402

VMEM = ("buffer_", "global_", "flat_", "scratch_")
WAITCNT = re.compile(r"(vmcnt|lgkmcnt|expcnt)\((\d+)\)")
FULL_WAIT = ("s_swappc_b64", "s_setpc_b64", "s_endpgm")


def regs(text: str):
    """VGPRs (ints) and SGPRs ('s<k>', 'vcc', ...) of an operand string."""
    return {("v", r) for r in H.vregs(text)} | {("s", r) for r in H.sregs(text) if r not in ("exec", "m0")}


def classify(mn: str, ops: str):
    """(counter kinds, destination registers) of a load-like instruction; ((), set()) otherwise.
    kinds: 'ds', 'smem', 'vm' (flat ops count on both vmcnt and lgkmcnt)."""
    o = H.operands(ops)
    if mn.startswith("ds_"):
        returns = mn.startswith(("ds_read", "ds_load")) or "_rtn" in mn or mn.startswith(("ds_swizzle", "ds_permute",
                                                                                         "ds_bpermute", "ds_consume",
                                                                                         "ds_append"))
        dst = regs(o[0].split()[0]) if returns and o else set()
        return ("ds",), dst
    if mn.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_memtime", "s_memrealtime", "s_dcache")):
        dst = regs(o[0].split()[0]) if o and not mn.startswith("s_dcache") else set()
        return ("smem",), dst
    if mn.startswith(VMEM):
        loads = "load" in mn or ("atomic" in mn and re.search(r"\b(glc|sc0)\b", ops) is not None)
        lds = "_lds" in mn or re.search(r"\blds\b", ops) is not None
        dst = regs(o[0].split()[0]) if loads and not lds and o else set()
        kinds = ("vm", "ds") if mn.startswith("flat_") else ("vm",)
        return kinds, dst
    return (), set()


def reads_writes(mn: str, ops: str):
    """Every register an instruction names (operands of either direction)."""
    return regs(" ".join(H.operands(ops)))


def apply_wait(state, ops):
    ds, smem, vm = state
    for kind, n in WAITCNT.findall(ops):
        n = int(n)
        if kind == "lgkmcnt":
            ds = ds[len(ds) - n:] if n < len(ds) else ds
            if n == 0:
                ds, smem = (), ()
        elif kind == "vmcnt":
            vm = vm[len(vm) - n:] if n < len(vm) else vm
    return ds, smem, vm


def merge(a, b):
    def m(x, y):
        n = max(len(x), len(y))
        x = (frozenset(),) * (n - len(x)) + x
        y = (frozenset(),) * (n - len(y)) + y
        return tuple(p | q for p, q in zip(x, y))
    return tuple(m(x, y) for x, y in zip(a, b))


def analyse(insts):
    """[(addr, text, conflicting registers, 'ds'|'smem'|'vm', load text)] for one function."""
    base = waitloops.base_of(insts)
    index = {a: k for k, (a, _, _) in enumerate(insts)}
    succ = {k: [] for k in range(len(insts))}
    leaders = {0}
    for k, (a, mn, ops) in enumerate(insts):
        if mn.startswith(("s_branch", "s_cbranch")):
            m = H.TARGET.search(ops)
            if m:
                tgt = base + int(m.group(2), 16) if m.group(2) else base
                if tgt in index:
                    succ[k].append(index[tgt])
                    leaders.add(index[tgt])
            leaders.add(k + 1)
        if k + 1 < len(insts) and mn not in H.NO_FALLTHROUGH:
            succ[k].append(k + 1)
    leaders = sorted(x for x in leaders if x < len(insts))
    block_of, blocks = {}, []
    for b, s in enumerate(leaders):
        e = leaders[b + 1] if b + 1 < len(leaders) else len(insts)
        blocks.append((s, e))
        for k in range(s, e):
            block_of[k] = b
    empty = ((), (), ())
    state_in = {0: empty}
    work = [0]
    loads = {}  # register set -> load text (diagnostics)
    bad = {}
    while work:
        b = work.pop()
        st = state_in[b]
        s, e = blocks[b]
        for k in range(s, e):
            a, mn, ops = insts[k]
            if mn == "s_waitcnt":
                st = apply_wait(st, ops)
                continue
            if mn in FULL_WAIT:
                st = empty
                continue
            kinds, dst = classify(mn, ops)
            used = reads_writes(mn, ops)
            if kinds:
                # a load's own destination may repeat an outstanding one of its kind (in-order returns)
                src_used = used - dst
            else:
                src_used = used
            ds, smem, vm = st
            for name, lst in (("ds", ds), ("smem", smem), ("vm", vm)):
                for ent in lst:
                    hit = ent & (src_used if name in kinds else used)
                    if hit:
                        bad.setdefault(a, (a, f"{mn} {ops}".strip(), sorted(map(str, hit)), name,
                                           loads.get(ent, "?")))
            if kinds:
                ent = frozenset(dst)
                loads.setdefault(ent, f"{mn} {ops}".strip())
                if "ds" in kinds:
                    ds = ds + (ent,)
                if "smem" in kinds:
                    smem = smem + (ent,)
                if "vm" in kinds:
                    vm = vm + (ent,)
                st = (ds[-64:], smem[-64:], vm[-64:])
        for nk in succ[e - 1] if e > s else []:
            nb = block_of[nk]
            new = st if nb not in state_in else merge(state_in[nb], st)
            if state_in.get(nb) != new:
                state_in[nb] = new
                work.append(nb)
    return sorted(bad.values())


def _analyse_item(item):
    return item[0], analyse(item[1])


def scan(so: Path, prefixes=None, workers=1):
    """{function: [early uses]}; workers > 1 analyses functions in that many processes."""
    items = [(name, insts) for name, insts in waitloops.functions(waitloops.disassemble(so)).items()
             if not prefixes or name.startswith(prefixes)]
    if workers <= 1:
        return dict(map(_analyse_item, items))
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor

    items.sort(key=lambda it: -len(it[1]))  # largest first: the long kernels set the wall time
    # spawned workers: a forked child would inherit the HIP runtime a loaded libmsa.so started in this
    # process, and the parent then faulted at interpreter exit (the CPU suite's exit status 139)
    with ProcessPoolExecutor(workers, mp_context=multiprocessing.get_context("spawn")) as ex:
        return dict(ex.map(_analyse_item, items, chunksize=1))


if __name__ == "__main__":
    so = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parent.parent / \
        "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    total = 0
    for name, bad in sorted(scan(so, workers=8).items()):
        total += len(bad)
        if bad:
            print(f"{len(bad):4d} early uses  {name[:110]}")
            for a, t, r, kind, ld in bad[:5]:
                print(f"        @{a:#x} {t[:60]:60s} {r} <- {kind}: {ld[:60]}")
    print(f"total early uses: {total}")
