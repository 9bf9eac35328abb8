"""Wait loops of libmsa.so's gfx950 code object (spin-wait loops = loops containing s_sleep), and how each
loops back: a wave-uniform back-edge (s_branch / s_cbranch_scc* / s_cbranch_vcc*) or an exec-mask one
(s_cbranch_execz / s_cbranch_execnz: the loop's control flow became divergent -- the hang class of rounds 3
and 4).  Used by tests/test_host.py::test_wait_loops_are_wave_uniform; run alone it prints a table.

    python scripts/waitloops.py [path/to/libmsa.so]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
INS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(<.*>)?")
FUN = re.compile(r"^([0-9a-f]+) <(.+)>:$")
BR = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>|<([^>]+)>")


def disassemble(so: Path) -> str:
    with tempfile.TemporaryDirectory() as td:
        fat, co = Path(td) / "fat.bin", Path(td) / "co.o"
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(so), str(fat) + ".elf"],
                       check=True)  # (an output file: without one objcopy rewrites the library in place)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--type=o", f"--targets={TARGET}", f"--input={fat}",
                        f"--output={co}", "--unbundle"], check=True)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                              capture_output=True, text=True).stdout


def functions(text: str):
    """{name: [(addr, mnemonic, operands), ...]}"""
    out, cur, base = {}, None, 0
    for ln in text.splitlines():
        mf = FUN.match(ln)
        if mf:
            cur = mf.group(2)
            base = int(mf.group(1), 16)
            out[cur] = []
            continue
        if cur is None:
            continue
        mi = INS.match(ln)
        if mi:
            out[cur].append((int(mi.group(3), 16), mi.group(1), mi.group(2) + " " + (mi.group(4) or "")))
    return out


def base_of(insts):
    return insts[0][0] if insts else 0


def wait_loops(insts):
    """Innermost spin-wait loops: for every s_sleep, the smallest range [target, branch] closed by a backward
    branch around it.  Returns [(back_edge_mnemonic, lo, hi, exec_writes_inside)] (one per distinct loop)."""
    base = base_of(insts)
    backs = []
    for a, mn, ops in insts:
        if not mn.startswith(("s_branch", "s_cbranch")):
            continue
        m = re.search(r"<(.+?)(?:\+0x([0-9a-f]+))?>", ops)
        if not m:
            continue
        tgt = base + int(m.group(2), 16) if m.group(2) else base
        if tgt < a:
            backs.append((a, tgt, mn))
    loops = {}
    for s_, mn_, _ in insts:
        if mn_ != "s_sleep":
            continue
        enc = [(a - t, a, t, mn) for a, t, mn in backs if t <= s_ <= a]
        if not enc:
            continue
        _, a, t, mn = min(enc)
        if (t, a) in loops:
            continue
        execw = any(t <= b <= a and (o.split(",")[0].strip() == "exec" or "saveexec" in mn2) for b, mn2, o in insts)
        loops[(t, a)] = (mn, t, a, execw)
    return list(loops.values())


EXEC_BR = ("s_cbranch_execz", "s_cbranch_execnz")


def violations(insts):
    """Exec-mask control of a wait loop: a backward s_cbranch_exec* inside it (the loop closes on the exec
    mask: SI_LOOP's divergent-loop lowering, or an if whose join is the latch) or an s_cbranch_exec* that
    leaves it (a divergent exit).  Forward exec branches that stay inside the loop (if (lane == 0) ...
    regions) are fine."""
    base = base_of(insts)
    sleeps = [a for a, mn, _ in insts if mn == "s_sleep"]
    bad = []
    for mn, lo, hi, _ in wait_loops(insts):
        zs = [z for z in sleeps if lo <= z <= hi]
        for a, m2, o in insts:
            if not (lo <= a <= hi) or m2 not in EXEC_BR:
                continue
            mt = re.search(r"<(.+?)(?:\+0x([0-9a-f]+))?>", o)
            tgt = base + int(mt.group(2), 16) if mt and mt.group(2) else base
            # an exit of the wait loop, or a back-edge around one of its sleeps (nested bounded loops
            # without a sleep -- a lane-strided copy -- are not wait loops)
            if not (lo <= tgt <= hi) or (tgt <= a and any(tgt <= z <= a for z in zs)):
                bad.append(dict(loop=(lo, hi), branch=m2, at=a, target=tgt))
    return bad


def scan(so: Path, prefixes=None):
    out = {}
    for name, insts in functions(disassemble(so)).items():
        if prefixes and not name.startswith(prefixes):
            continue
        out[name] = dict(loops=len(wait_loops(insts)), bad=violations(insts))
    return out


if __name__ == "__main__":
    so = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parent.parent / \
        "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    for name, r in sorted(scan(so).items()):
        if r["loops"]:
            print(f"{r['loops']:3d} wait loops, {len(r['bad']):2d} exec-controlled  {name[:100]}")
            for b in r["bad"]:
                print(f"      {b['branch']} at {b['at']:#x} -> {b['target']:#x} in loop {b['loop'][0]:#x}..{b['loop'][1]:#x}")
