"""Per-kernel resources from libmsa.so's gfx950 code-object metadata (no recompilation): VGPRs, SGPRs,
scratch bytes per lane, spills, LDS.

    python scripts/kmeta.py [substring] [path/to/libmsa.so]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def kernels(so: Path):
    with tempfile.TemporaryDirectory() as td:
        fat, co = Path(td) / "fat.bin", Path(td) / "co.o"
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(so), str(fat) + ".elf"],
                       check=True)  # (an output file: without one objcopy rewrites the library in place)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fat}", f"--output={co}", "--unbundle"], check=True)
        txt = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                             text=True).stdout
    out, cur = [], None
    for ln in txt.splitlines():
        m = re.match(r"^\s+(-\s+)?\.(\w+):\s+(.*)$", ln)
        if not m:
            continue
        key, val = m.group(2), m.group(3).strip()
        if m.group(1) and key != "name" and cur is not None and key in cur:
            cur = None
        if key == "name" and (cur is None or "name" in cur):
            cur = {}
            out.append(cur)
        if cur is not None:
            cur.setdefault(key, val)
    return [k for k in out if "vgpr_count" in k]


if __name__ == "__main__":
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    so = Path(sys.argv[2]) if len(sys.argv) > 2 else Path(__file__).resolve().parent.parent / \
        "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    for k in kernels(so):
        if flt in k.get("name", ""):
            print(f"{k.get('vgpr_count','?'):>4} vgpr {k.get('sgpr_count','?'):>4} sgpr "
                  f"scratch {k.get('private_segment_fixed_size','?'):>4} vspill {k.get('vgpr_spill_count','?'):>3} "
                  f"lds {k.get('group_segment_fixed_size','?'):>5}  {k.get('name','?')[:100]}")
