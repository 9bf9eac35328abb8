"""Host-side logic on CPU: the C-ABI library, stripe geometry, SW oracle vs brute force."""
import ctypes as C
import os
import re
import sys

import numpy as np
import pytest

from conftest import ROOT


def test_library_exports_every_header_symbol():
    """libmsa.so loads and exports every function include/msa.h declares (no compute calls)."""
    from cse305_parallel_sequence_alignment_amd import _lib as LB

    hdr = (ROOT / "include" / "msa.h").read_text()
    declared = set(re.findall(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(msa_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    L = LB.lib()
    for name in sorted(declared):
        assert hasattr(L, name), f"libmsa.so does not export {name}"
    assert declared == set(LB.EXPORTED)


def test_status_strings_and_version():
    from cse305_parallel_sequence_alignment_amd import _lib as LB

    L = LB.lib()
    assert L.msa_version() >= 1
    for code in LB.STATUS:
        assert L.msa_status_string(code)


def test_encode_pair_alphabet():
    """msa_encode_pair: first-seen symbol codes, > 8 distinct symbols rejected (pure host code)."""
    from cse305_parallel_sequence_alignment_amd import _lib as LB

    L = LB.lib()
    a, b = C.create_string_buffer(16), C.create_string_buffer(16)
    assert L.msa_encode_pair(b"ACGT", 4, b"GGTA", 4, a, b) == 0
    assert list(a.raw[:4]) == [0, 1, 2, 3] and list(b.raw[:4]) == [2, 2, 3, 0]
    assert L.msa_encode_pair(b"ABCDEFGHI", 9, b"A", 1, a, b) == -2


def test_no_cpu_fallback_without_gpu():
    """On a machine without gfx950 the product path fails loudly (MSA_ERR_NODEV), it never computes on the CPU."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cse305_parallel_sequence_alignment_amd import api, MsaError

    with pytest.raises(MsaError) as e:
        api.main_alignment_text(b"-AGGA", b"-AGTGC", 4, 5, 3, 1, 2)
    assert e.value.status == -4


def test_stripe_phases_cover_every_cell():
    """Stripe s (rows 64s+1..64s+64) runs 16*phases anti-diagonal steps covering columns jlo..jhi of each row."""
    from cse305_parallel_sequence_alignment_amd.plan import jhi_of, jlo_of, stripe_geom

    for (m, n, band, ks) in [(1, 1, -1, 16), (64, 64, -1, 16), (65, 100, -1, 32), (700, 650, -1, 16), (700, 650, -1, 32),
                             (1000, 1000, 32, 16), (500, 900, 512, 32)]:
        S = (m + 63) // 64
        for s in range(S):
            cs, P = stripe_geom(s, m, n, band, ks)
            for r in range(min(64, m - 64 * s)):
                i = 64 * s + r + 1
                jl, jh = jlo_of(i, band), jhi_of(i, n, band)
                if jl > jh:
                    continue
                # lane r processes column cs + t - r at step t
                assert cs + 0 - r <= jl and cs + ks * P - 1 - r >= jh


def brute_sw(A, B, ma, mi, go, ge):
    m, n = len(A), len(B)
    NEG = -(1 << 30)
    H = np.zeros((m + 1, n + 1), dtype=np.int64)
    E = np.full((m + 1, n + 1), NEG, dtype=np.int64)
    F = np.full((m + 1, n + 1), NEG, dtype=np.int64)
    best, end = 0, (0, 0)
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            E[i, j] = max(H[i, j - 1] - go, E[i, j - 1] - ge)
            F[i, j] = max(H[i - 1, j] - go, F[i - 1, j] - ge)
            s = ma if A[i - 1] == B[j - 1] else mi
            H[i, j] = max(0, H[i - 1, j - 1] + s, E[i, j], F[i, j])
            if H[i, j] > best:
                best, end = int(H[i, j]), (i, j)
    return best, end, H


@pytest.mark.parametrize("params", [(1, 0, 1, 1), (2, -1, 1, 1), (2, -3, 5, 2), (1, -1, 3, 1)])
def test_oracle_sw_vs_brute_force(oracle, params):
    rng = np.random.default_rng(5)
    for _ in range(6):
        m, n = rng.integers(1, 40, size=2)
        A = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), m).tobytes()
        B = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()
        best, end, H = brute_sw(A, B, *params)
        o = oracle.sw(A, B, *params, want_h=True, want_tb=True)
        assert o["score"] == best and tuple(o["end"]) == end
        assert np.array_equal(o["H"], H.astype(np.int32))
        # the traceback re-scores to the optimum
        i, j = o["beg"][0] - 1, o["beg"][1] - 1  # beg is the 1-based first aligned cell
        sc, ext_a, ext_b = 0, False, False
        for num, op in re.findall(r"(\d+)([MID])", o["cigar"]):
            for _ in range(int(num)):
                if op == "M":
                    sc += params[0] if A[i] == B[j] else params[1]
                    i, j, ext_a, ext_b = i + 1, j + 1, False, False
                elif op == "I":  # consumes A only (B is the reference, SAM convention)
                    sc -= params[3] if ext_a else params[2]
                    i, ext_a, ext_b = i + 1, True, False
                else:
                    sc -= params[3] if ext_b else params[2]
                    j, ext_a, ext_b = j + 1, False, True
        assert sc == best and (i, j) == tuple(end)


def test_checksum_matches_numpy_restatement(oracle):
    rng = np.random.default_rng(1)
    H = rng.integers(-50, 200, size=(33, 47)).astype(np.int32)
    w = oracle.mix_matrix(32, 46)
    with np.errstate(over="ignore"):
        want = int((w[1:, 1:] * H[1:, 1:].astype(np.uint32).astype(np.uint64)).sum(dtype=np.uint64))
    assert oracle.checksum_h(H) == want


def test_banded_equals_full_when_band_covers(oracle):
    """NW banded (Gotoh, reference scoring) with a band wider than the matrix == main_alignment's score."""
    rng = np.random.default_rng(2)
    for _ in range(4):
        m, n = rng.integers(5, 60, size=2)
        A = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), m).tobytes()
        B = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()
        _, full = oracle.main_alignment_text(A, B, 1.0, 2.0)
        assert oracle.banded_ref(A, B, max(m, n) + 2, 1.0, 2.0) == full


def test_compat_library_exports_reference_symbol():
    """libmsa_compat.so exports main_alignment_function with the reference's C++ mangling
    (alignment_algorithm/main_alignment.h:38 -> _Z23main_alignment_functionPcS_mmmdd)."""
    lib = ROOT / "cse305_parallel_sequence_alignment_amd" / "libmsa_compat.so"
    assert lib.exists(), "build libmsa_compat.so (make -C cse305_parallel_sequence_alignment_amd/csrc)"
    L = C.CDLL(str(lib))
    assert hasattr(L, "_Z23main_alignment_functionPcS_mmmdd")


SUBPROBLEM_SYMBOLS = [
    "_ZN10Subproblem14compute_tablesEv", "_ZN10Subproblem19non_parallel_tablesEv", "_ZN10Subproblem11compute_rowEm",
    "_ZN10Subproblem14find_alignmentEv", "_ZN10Subproblem15print_alignmentEv",
    "_ZN10Subproblem24ComputeFirstRowMapThreadEPS_mm", "_ZN10Subproblem21ComputeRowMapThread13EPS_mmm",
    "_ZN10Subproblem21ComputeOmegaMapThreadEPS_mmmRSt6vectorIdSaIdEE",
    "_ZN10Subproblem20ComputeRowMapThread2EPS_mmmRSt6vectorIdSaIdEE",
]


def test_compat_library_exports_subproblem_members():
    """libmsa_compat.so defines every out-of-line member of the reference's class Subproblem
    (alignment_algorithm/subproblem_alignment.h:76-95) with the reference's C++ mangling, and the
    test driver built against include/subproblem_alignment_compat.h links."""
    lib = ROOT / "cse305_parallel_sequence_alignment_amd" / "libmsa_compat.so"
    L = C.CDLL(str(lib))
    for sym in SUBPROBLEM_SYMBOLS:
        assert hasattr(L, sym), sym
    assert (ROOT / "tests" / "cpp" / "subproblem_driver").exists(), "make -C tests/cpp"


# main_alignment.h:17-38 and partial.h:23-41 with the reference's C++ manglings (types as declared by the
# reference headers; `align` is struct alignment_point, queue_indices struct parallel_prefix_queue_element)
MAIN_ALIGNMENT_SYMBOLS = [
    "_Z25OptimalAlignmentMapThreadPcS_mmmmmiiddRP15alignment_pointS2_", "_Z11print_alignP15alignment_point",
    "_Z18PrefixSumMapThreadRSt6vectorIlSaIlEElP29parallel_prefix_queue_element",
    "_Z19PrefixInitMapThreadRSt6vectorIlSaIlEES2_R29parallel_prefix_queue_element",
    "_Z14ParallelPrefixmRSt6vectorIlSaIlEES2_",
    "_Z21ComputeOmegaMapThreadN9__gnu_cxx17__normal_iteratorIP15alignment_pointSt6vectorIS1_SaIS1_EEEES6_mmmRS3_IlSaIlEEl",
    "_Z22compute_omega_parallelRSt6vectorI15alignment_pointSaIS0_EEmmmmRS_IlSaIlEE", "_Z17assign_processorsll",
    "_Z17optimal_alignmentPcS_St6vectorI15alignment_pointSaIS1_EEmmmdd", "_Z23main_alignment_functionPcS_mmmdd",
]
PARTIAL_SYMBOLS = [
    "_Z5scorecc", "_Z16initializeTablesRSt6vectorIS_IiSaIiEESaIS1_EES4_S4_mmddi",
    "_Z23initializeReverseTablesRSt6vectorIS_IiSaIiEESaIS1_EES4_S4_mmddi",
    "_Z18fillTablesParallelPKcS0_mmRSt6vectorIS1_IiSaIiEESaIS3_EES6_S6_ddm",
    "_Z25fillReverseTablesParallelPKcS0_mmRSt6vectorIS1_IiSaIiEESaIS3_EES6_S6_ddm",
    "_Z21findPartitionParallelRKSt6vectorIS_IiSaIiEESaIS1_EES5_S5_S5_S5_S5_mmmd",
    "_Z36findPartialBalancedPartitionParallelPKcS0_mmmddiiRSt6vectorI15alignment_pointSaIS2_EE",
]


def test_compat_library_exports_main_alignment_and_partial_api():
    """libmsa_compat.so defines every function alignment_algorithm/main_alignment.h:17-38 and
    sequence_alignment/partial.h:23-41 declare (extractPartitions aside: the reference defines no body),
    with the reference's C++ manglings; the drivers compiled against the reference's own headers
    (oracle/_ref/*_driver_refhdr, where /root/reference exists) linked against it."""
    lib = ROOT / "cse305_parallel_sequence_alignment_amd" / "libmsa_compat.so"
    L = C.CDLL(str(lib))
    for sym in MAIN_ALIGNMENT_SYMBOLS + PARTIAL_SYMBOLS:
        assert hasattr(L, sym), sym
    for d in ("optimal_driver", "partial_driver"):
        assert (ROOT / "tests" / "cpp" / d).exists(), "make -C tests/cpp"


def _drivers(name):
    out = [ROOT / "tests" / "cpp" / name]
    ref = ROOT / "oracle" / "_ref" / f"{name}_refhdr"
    return out + ([ref] if ref.exists() else [])


def test_cpp_scheduler_helpers_and_score_on_host():
    """The host-only parts of the two C++ APIs through both driver builds (no GPU needed): the scheduler
    bookkeeping of main_alignment.cpp:158-200 (omega, ParallelPrefix, assign_processors, the block bodies)
    and partial.cpp:9-11's score; a GPU entry point without a GPU throws (no CPU fallback)."""
    import subprocess

    cases = "sched 4 40 40 5 0 0 -1 1 13 3 1 23 3 40 37 1 40 40 1\nsched 3 10 7 3 0 0 -1 4 2 2 10 7 1\n" \
            "opt 1.0 2.0 4 4 5 AGGA AGTGC 2 0 0 -1 4 5 1\n"
    want = ("OMEGA 2 1 4 1\nSUMS 2 3 7 8\nPROCS 1 1 2 1\nOMEGA1 2 1 4 1\nINIT 2 3 7 8 | 8\nADD7 9 10 14 15\nEND_CASE\n"
            # (4,2): ceil(4/(10/3)) = 2, ceil(2/(7/3)) = 1; (6,5): ceil(1.8) = 2, ceil(2.14) = 3
            "OMEGA 2 3\nSUMS 2 5\nPROCS 1 2\nOMEGA1 2 3\nINIT 2 5 | 5\nADD7 9 12\nEND_CASE\n")
    for drv in _drivers("optimal_driver"):
        r = subprocess.run([str(drv)], input=cases, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert r.stdout.startswith(want), (drv.name, r.stdout)
        assert "ERROR optimal_alignment: no gfx950 device" in r.stdout or "ERROR" not in r.stdout
    for drv in _drivers("partial_driver"):
        r = subprocess.run([str(drv)], input="score A A\nscore A C\nscore T G\n", capture_output=True, text=True,
                           timeout=60)
        assert r.returncode == 0, r.stderr
        assert r.stdout == "SCORE 0\nEND_CASE\nSCORE 1\nEND_CASE\nSCORE 1\nEND_CASE\n", drv.name


def _similarity_reference_loop(s1: bytes, s2: bytes, T: int) -> float:
    """pull_data.cpp:97-125 transcribed as loops (chunking, remainder on chunk T-1, / max length)."""
    L = min(len(s1), len(s2))
    chunk = L // T
    score = 0
    for i in range(L // chunk):
        start = i * chunk
        end = start + chunk + (L % T if i == T - 1 else 0)
        score += sum(1 for k in range(start, end) if s1[k] == s2[k])
    return score / max(len(s1), len(s2))


def test_harness_similarity_and_reader():
    """Build-owned harness (harness.py): sequence_similarity follows the reference's chunking
    (positions double-counted when L // chunk > T) and read_and_store_sequences fills the lists."""
    from cse305_parallel_sequence_alignment_amd import harness

    names, seqs = [], []
    assert harness.read_and_store_sequences(names, seqs) == 0
    assert len(names) == len(seqs) == 20
    for (a, b) in ((0, 1), (3, 4), (5, 17)):
        for T in (1, 3, 7, 16, 64):
            s1, s2 = seqs[a][:5000 + 37 * T], seqs[b][:4000]
            assert harness.sequence_similarity(s1, s2, T) == _similarity_reference_loop(s1, s2, T)
    assert harness.sequence_similarity(b"ACGTACGTAC", b"ACGAACGTAA", 4) == _similarity_reference_loop(
        b"ACGTACGTAC", b"ACGAACGTAA", 4)


def _waitloops():
    import importlib.util

    spec = importlib.util.spec_from_file_location("waitloops", ROOT / "scripts" / "waitloops.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_wait_loop_detector_flags_exec_controlled_loops():
    """The detector itself, on a hand-written disassembly: a spin loop closed by s_cbranch_execnz (the
    divergent-loop lowering) is flagged, the same loop closed by s_cbranch_scc1 is not, and a lane-strided
    inner loop without a sleep does not count."""
    W = _waitloops()

    def fn(back):
        return [(0x100, "s_nop", "0 "), (0x104, "global_load_dwordx2", "v[0:1], v[2:3], off "),
                (0x108, "v_cmp_ne_u32_e32", "vcc, s4, v1 "), (0x10c, "s_sleep", "1 "),
                (0x110, "s_and_b64", "exec, exec, vcc "), (0x114, back, "-4 <f+0x4>"),
                (0x118, "s_endpgm", " ")]

    bad = W.violations(fn("s_cbranch_execnz"))
    assert len(bad) == 1 and bad[0]["branch"] == "s_cbranch_execnz"
    assert W.violations(fn("s_cbranch_scc1")) == []
    inner = [(0x100, "s_sleep", "1 "), (0x104, "v_add_u32_e32", "v0, 64, v0 "),
             (0x108, "s_cbranch_execnz", "-2 <f+0x4>"), (0x10c, "s_cbranch_scc1", "-4 <f+0x0>")]
    assert W.violations(inner) == []


def test_wait_loops_are_wave_uniform():
    """Every spin-wait loop (a loop around an s_sleep) of every kernel in libmsa.so's gfx950 code object
    closes and exits on scalar state (s_branch / s_cbranch_scc* / s_cbranch_vcc*), never on the exec
    mask.  Rounds 3 and 4 each hung a GPU run when codegen turned such a loop divergent (an inlined
    block body; a spin-limit error store inside the loop); this guards the flow kernels, the band
    kernel, the pass-2 block bodies and the stripe kernel's loader against it from the CPU suite."""
    W = _waitloops()
    so = ROOT / "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    if not so.exists():
        pytest.skip("libmsa.so not built")
    res = W.scan(so)
    with_loops = {k: v for k, v in res.items() if v["loops"]}
    for prefix in ("_ZN3msa11flow_kernel", "_ZN3msa11band_kernel", "_ZN3msa13stripe_kernel",
                   "_ZN3msa12cflow_kernel",
                   "_ZN3msa10fill_block", "_ZN3msa14fill_block_aff", "_ZN3msa14fill_block_got"):
        assert any(k.startswith(prefix) for k in with_loops), f"no wait loop found in {prefix}*"
    bad = {k: v["bad"] for k, v in with_loops.items() if v["bad"]}
    assert not bad, f"exec-mask controlled wait loops: {bad}"


def _isa_hazards():
    import importlib.util

    sys.path.insert(0, str(ROOT / "scripts"))
    spec = importlib.util.spec_from_file_location("isa_hazards", ROOT / "scripts" / "isa_hazards.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_asm_hazard_detector():
    """The detector on hand-written code.  DPP: one instruction after the VALU write of its source is short
    (1 wait state of the 2 gfx950 needs); an `s_nop 1`, or two instructions, in between make it clean; a
    write reaching the DPP through a branch to its block counts; so does a write of the DPP's destination
    (the `old` value of lanes with no source lane); SGPR / VCC writes do not.  The other classes: M0 ->
    LDS add-TID (1), VALU SGPR write -> VMEM address (5), -> v_readlane lane select (4), v_cmpx -> DPP (5)."""
    H = _isa_hazards()
    dpp = (0x10c, "v_mov_b32_dpp", "v5, v1 wave_shr:1 row_mask:0xf bank_mask:0xf ")

    def fn(*mid):
        return [(0x100, "v_pk_max_i16", "v1, v1, v24 ")] + [(0x104 + 4 * k, mn, o) for k, (mn, o) in
                                                               enumerate(mid)] + [dpp, (0x200, "s_endpgm", " ")]

    bad = H.hazards(fn(("v_pk_add_u16", "v2, v3, v4 ")))
    assert [(b[0], b[5], b[6]) for b in bad] == [("dpp_vgpr", 1, [1])]
    assert H.hazards(fn(("v_pk_add_u16", "v2, v3, v4 "), ("s_nop", "0 "))) == []
    assert H.hazards(fn(("s_nop", "1 "))) == []
    assert len(H.hazards(fn(("s_nop", "0 ")))) == 1
    assert H.hazards(fn(("v_cmp_gt_i32_e32", "vcc, v1, v2 "), ("v_readfirstlane_b32", "s4, v1 "))) == []
    # destination written one instruction before the DPP
    assert len(H.hazards([(0x100, "v_add_u32_e32", "v5, 1, v5 "), (0x104, "s_nop", "0 "), (0x108,) + dpp[1:]])) == 1
    # a branch from a block ending in the write, over clean fall-through code
    br = [(0x100, "v_mov_b32_e32", "v1, 0 "), (0x104, "s_cbranch_scc1", "4 <f+0x18>"),
          (0x108, "s_nop", "4 "), (0x10c, "s_nop", "4 "), (0x110, "s_branch", "3 <f+0x20>"),
          (0x114, "s_nop", "0 "), (0x118,) + dpp[1:], (0x11c, "s_endpgm", " ")]
    assert len(H.hazards(br)) == 1
    # the other classes, short and padded
    m0 = [(0x100, "s_mov_b32", "m0, s3 "), (0x104, "ds_write_addtid_b32", "v1 offset:0 ")]
    assert [b[0] for b in H.hazards(m0)] == ["m0_lds"]
    assert H.hazards([m0[0], (0x104, "s_nop", "0 "), (0x108,) + m0[1][1:]]) == []
    vm = [(0x100, "v_readfirstlane_b32", "s4, v1 "), (0x104, "s_nop", "3 "), (0x108, "global_load_dword", "v2, v3, s[4:5] ")]
    assert [b[0] for b in H.hazards(vm)] == ["sgpr_vmem"]
    assert H.hazards([vm[0], (0x104, "s_nop", "4 "), vm[2]]) == []
    ls = [(0x100, "v_readfirstlane_b32", "s4, v1 "), (0x104, "s_nop", "2 "), (0x108, "v_readlane_b32", "s6, v2, s4 ")]
    assert [b[0] for b in H.hazards(ls)] == ["lane_select"]
    assert H.hazards([ls[0], (0x104, "s_nop", "3 "), ls[2]]) == []
    cx = [(0x100, "v_cmpx_gt_i32_e32", "vcc, v1, v2 "), (0x104, "s_nop", "3 "), (0x108,) + dpp[1:]]
    assert [b[0] for b in H.hazards(cx)] == ["dpp_exec"]


def test_asm_hazards_have_their_wait_states():
    """Every kernel and device function in libmsa.so's gfx950 code object gives each software-managed
    hazard its wait states on every control-flow path: VALU-write -> DPP-read (2), VALU EXEC write -> DPP
    (5), M0 -> LDS add-TID / LDS-DMA (1), VALU SGPR write -> VMEM (5) and -> lane select (4).  hipcc pads
    what it emits; inline asm is not padded -- round 5's cflow_kernel had 47 DPPs reading X one wait state
    after the v_pk_max_i16 that wrote it, correct only by issue timing."""
    H = _isa_hazards()
    so = ROOT / "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    if not so.exists():
        pytest.skip("libmsa.so not built")
    res = H.scan(so)
    for prefix in ("_ZN3msa11flow_kernel", "_ZN3msa11band_kernel", "_ZN3msa13stripe_kernel",
                   "_ZN3msa12cflow_kernel", "_ZN3msa14fill_block_aff", "_ZN3msa14fill_block_got"):
        assert any(k.startswith(prefix) and v[0].get("dpp_vgpr") for k, v in res.items()), f"no DPP in {prefix}*"
    assert any(v[0].get("m0_lds") for k, v in res.items() if "traceback_kernel" in k), "no LDS-DMA in the walk"
    bad = {k: v[1][:3] for k, v in res.items() if v[1]}
    assert not bad, f"hazards short of their wait states: {bad}"


def test_async_loads_are_waited_for():
    """No instruction of libmsa.so's gfx950 code object reads or overwrites the destination of an LDS or
    global load before an s_waitcnt covers it (scripts/isa_async.py: dataflow over every function's
    control flow, DS in order / SMEM out of order on lgkmcnt, VMEM in order on vmcnt).  The flow, band and
    cflow kernels issue their ring / counter reads as inline asm with explicit waits, which the compiler
    does not count: a register copy or spill it placed between such a read and its wait would read a
    value that has not landed."""
    sys.path.insert(0, str(ROOT / "scripts"))
    import isa_async as A  # (an importable module: the scan's worker processes unpickle its functions)

    ins = [(0x100, "ds_read_b128", "v[4:7], v1 offset:16 "), (0x104, "v_mov_b32_e32", "v8, v5 "),
           (0x108, "s_waitcnt", "lgkmcnt(0) "), (0x10c, "v_mov_b32_e32", "v9, v5 ")]
    assert [b[0] for b in A.analyse(ins)] == [0x104]  # the detector itself
    ins = [(0x100, "s_load_dwordx2", "s[4:5], s[0:1], 0x0 "), (0x104, "ds_read_b32", "v10, v1 "),
           (0x108, "s_waitcnt", "lgkmcnt(1) "), (0x10c, "v_mov_b32_e32", "v9, v10 ")]
    assert [b[0] for b in A.analyse(ins)] == [0x10c]  # SMEM may complete first: the DS read may not have
    so = ROOT / "cse305_parallel_sequence_alignment_amd" / "libmsa.so"
    if not so.exists():
        pytest.skip("libmsa.so not built")
    res = A.scan(so, prefixes=("_ZN3msa",), workers=min(8, os.cpu_count() or 1))
    assert any(k.startswith("_ZN3msa12cflow_kernel") for k in res)
    bad = {k: v[:3] for k, v in res.items() if v}
    assert not bad, f"async results used before their wait: {bad}"


def test_oracle_under_sanitizers():
    """The CPU oracle (oracle/msa_oracle.c, oracle/cpu_rowsweep.cpp) built with AddressSanitizer and
    UndefinedBehaviorSanitizer (every UB report aborts: partial.cpp's wrap semantics must be restated
    without signed overflow), then tests/test_oracle_golden.py against it in a child process with the
    sanitizer runtimes preloaded -- all the reference-produced fixtures, the KATs and the live comparison
    with the reference's own code.  The multi-second at-size cases are left to the plain build."""
    import subprocess

    r = subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    gcc = lambda lib: subprocess.run(["gcc", f"-print-file-name={lib}"], capture_output=True,  # noqa: E731
                                     text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=f"{gcc('libasan.so')}:{gcc('libubsan.so')}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               MSA_ORACLE_DIR=str(ROOT / "oracle" / "_san"))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        str(ROOT / "tests" / "test_oracle_golden.py"), "-k",
                        "not at_size and not rowsweep_baseline_matches_oracle[8] and "
                        "not rowsweep_baseline_matches_oracle[3]"],
                       capture_output=True, text=True, env=env, cwd=str(ROOT), timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert " passed" in r.stdout and "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
