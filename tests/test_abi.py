"""CPU tier: the C-ABI library loads and exports every symbol include/sbce.h
declares; struct layouts agree between C (gcc) and the ctypes binding; argument
validation works without touching a GPU."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sbce.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(sbce_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points(sbce):
    assert _declared() == sorted(sbce._lib.EXPORTED)


def test_library_exports_every_declared_symbol(sbce):
    lib = sbce._lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.sbce_abi_version() == sbce._lib.SBCE_ABI_VERSION
    assert lib.sbce_strerror(-1)


def test_product_library_has_no_switches_and_ab_build_has_same_abi(sbce):
    """The product library reads no environment (no getenv import, sbce_debug_reload_env -1,
    the skip mask refused); the A/B build (csrc/sbce_internal.h SBCE_AB) exports the same
    C-ABI and reads its SBCE_* switches."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    def undef(path):
        out = subprocess.run([nm, "-D", "--undefined-only", path], capture_output=True,
                             text=True, check=True).stdout
        return {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}
    assert "getenv" not in undef(sbce._lib.LIB_PATH)
    assert "getenv" in undef(sbce._lib.AB_LIB_PATH)
    prod, ab = sbce._lib.load(), sbce._lib.load_ab()
    assert prod is not ab
    for name in _declared():
        assert hasattr(ab, name), name
    assert ab.sbce_abi_version() == sbce._lib.SBCE_ABI_VERSION
    assert prod.sbce_debug_reload_env() == -1
    assert prod.sbce_debug_chol_skip(8) == -2
    assert ab.sbce_debug_reload_env() == 0         # no switch set here: defaults


def test_struct_layout_matches_c(sbce, tmp_path):
    """Compile a probe against include/sbce.h with gcc and compare sizes/offsets."""
    probe = tmp_path / "probe.c"
    probe.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "sbce.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(sbce_dims), offsetof(sbce_dims, varn),
         sizeof(sbce_ptrs), offsetof(sbce_ptrs, workspace_bytes), offsetof(sbce_ptrs, x_dest),
         offsetof(sbce_dims, partition_r), offsetof(sbce_dims, varx), offsetof(sbce_ptrs, varn_t));
  return 0;
}''')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(probe), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    L = sbce._lib
    assert [int(v) for v in out] == [ctypes.sizeof(L.Dims), L.Dims.varn.offset,
                                     ctypes.sizeof(L.Ptrs), L.Ptrs.workspace_bytes.offset,
                                     L.Ptrs.x_dest.offset, L.Dims.partition_r.offset,
                                     L.Dims.varx.offset, L.Ptrs.varn_t.offset]


def test_integration_snippet_matches_abi(sbce):
    """INTEGRATION.md's raw ctypes binding (section 3) is what a maintainer copies: its
    struct definitions must equal _lib.py's, field by field, and therefore the C layout
    (test_struct_layout_matches_c), or sbce_em reads past the caller's structs."""
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = md[md.index("## 3. Raw ctypes binding"):md.index("## 4.")]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    # the class definitions and the ABI version only (the rest needs a GPU and buffers)
    head = code[:code.index("lib = ctypes.CDLL")]
    ns = {}
    exec(head, ns)
    L = sbce._lib
    assert ns["SBCE_ABI_VERSION"] == L.SBCE_ABI_VERSION
    for name in ("Dims", "Ptrs"):
        doc, lib = ns[name], getattr(L, name)
        assert [(f, t) for f, t in doc._fields_] == [(f, t) for f, t in lib._fields_], name
        assert ctypes.sizeof(doc) == ctypes.sizeof(lib)
    # every field the C header declares appears in the snippet, in order
    src = open(HEADER).read()
    for cname, pyname in (("sbce_dims", "Dims"), ("sbce_ptrs", "Ptrs")):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        cfields = re.findall(r"(\w+)\s*;", body)
        assert cfields == [f for f, _ in ns[pyname]._fields_], (cname, cfields)


def test_workspace_and_validation_without_gpu(sbce):
    L = sbce._lib
    lib = L.load()
    d = L.Dims(1000, 4, 4, 65, 16, 256, 16, 0, 0.1)
    n = L.workspace_bytes(d)
    Lw = 65 * 4
    expect = (1000 * 256 * 20 * 16 + 1000 * Lw * Lw * 16 + 1000 * Lw * 4 * 16
              + 1000 * 256 * 4 * 16                       # moments, R, rhs, shifted y
              + 1000 * 256 * (4 + 2 * 16 + 16 + 6 * 4) * 8  # E-step prep (H_eff, bounds,
                                                            # row-bound vectors)
              + (3 * 1000 * 256 + 32) * 4                   # sphere pass: sweep, enumeration and
                                                            # factorised-pass lists + counters
              + 1000 * 256 * 32 * 8                         # sphere pass: search-tree records
              + 1000 * 16 * 65 * 16 + 1000 * 16 * 16 * 16  # factored pilots psi', x' x'^H
              + 1000 * 4 + 1000 * 8                       # pilot flags, pivot thresholds
              + 1000 * Lw * 4 * 16                        # pilot part of B^H (once per run)
              + 1000 * 64 * 64 * 16                       # tiled factorisation: tile inverse
              + 1000 * Lw * Lw * 16 + 1000 * Lw * 4 * 16  # min-norm solve: C = G^H G, G^H B^H
              + 1000 * 4 + 1000 * 8                       # min-norm: extents, C's threshold
              + 1000 * Lw * 8                             # min-norm: Schur-complement diagonal
              + 1000 * Lw * 4 * 16 + 1000 * 4)            # min-norm: refinement residual, gate
    assert expect <= n <= expect + 16 * 256 + 4000
    # one solve mode (ABI 5): CHOL at L <= 512 carves neither the tile inverses nor the min-norm
    # regions; the min-norm solve needs all of them (= the any-mode size)
    chol = L.workspace_bytes(d, L.SBCE_SOLVE_CHOL)
    assert L.workspace_bytes(d, L.SBCE_SOLVE_CHOL_DROP) == chol
    assert L.workspace_bytes(d, L.SBCE_SOLVE_MINNORM) == n
    mn_only = (1000 * 64 * 64 * 16 + 1000 * Lw * Lw * 16 + 1000 * Lw * 4 * 16 + 1000 * 4
               + 1000 * 8 + 1000 * Lw * 8 + 1000 * Lw * 4 * 16 + 1000 * 4)
    assert 0 <= n - chol - mn_only <= 8 * 256
    # L > 512 (tiled factorisation): CHOL keeps the tile inverses
    big = L.Dims(4, 8, 8, 257, 32, 64, 16, 1, 0.1)
    nbig, cbig = L.workspace_bytes(big), L.workspace_bytes(big, L.SBCE_SOLVE_CHOL)
    Lb = 257 * 8
    assert 0 <= nbig - cbig - (4 * Lb * Lb * 16 + 2 * 4 * Lb * 8 * 16 + 2 * 4 * 4 + 4 * 8
                               + 4 * Lb * 8) <= 7 * 256
    assert lib.sbce_workspace_bytes_solve(ctypes.byref(d), 7, ctypes.byref(ctypes.c_size_t())) == -1
    bad = L.Dims(1, 9, 4, 65, 16, 256, 16, 0, 0.1)     # n_tx > 8
    nb = ctypes.c_size_t(0)
    assert lib.sbce_workspace_bytes(ctypes.byref(bad), ctypes.byref(nb)) == -1
    bad2 = L.Dims(1, 2, 2, 5, 4, 8, 4, 0, 0.0)         # varn must be > 0
    assert lib.sbce_workspace_bytes(ctypes.byref(bad2), ctypes.byref(nb)) == -1
    # null pointers are rejected before any HIP call
    p = L.Ptrs()
    assert lib.sbce_em(ctypes.byref(d), ctypes.byref(p), 1, 0, 0, None) == -1
    # a CHOL-sized workspace is too small for the min-norm solve (before any HIP call)
    p = L.Ptrs(*([256] * 11), 256, chol)
    assert lib.sbce_em(ctypes.byref(d), ctypes.byref(p), 1, 0, L.SBCE_SOLVE_MINNORM, None) == -4


def test_product_path_fails_loudly_without_gpu(sbce):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    d = {"Y_d": None}
    with pytest.raises(sbce.SbceUnavailable):
        sbce.em_batch(*(None,) * 5, 0.1, 1, None)
    del d


def test_oversized_problems_are_unsupported_without_gpu(sbce):
    """chol_supported: L <= 8192 (the tiled large-L path); larger systems are rejected with
    SBCE_EUNSUPPORTED before any pointer is dereferenced or HIP call made."""
    L = sbce._lib
    lib = L.load()
    big = L.Dims(2, 8, 4, 1025, 16, 64, 16, 1, 0.1)      # L = 1025 * 8 = 8200 > 8192
    p = L.Ptrs(*([16] * 12), 1 << 62)
    assert lib.sbce_em(ctypes.byref(big), ctypes.byref(p), 1, L.SBCE_ESTEP_PM_SOFT,
                       L.SBCE_SOLVE_CHOL, None) == -2
    assert lib.sbce_mstep(ctypes.byref(big), ctypes.byref(p), 16, 0, None, None, None) == -2
    ok = L.Dims(2, 8, 4, 1024, 16, 64, 16, 1, 0.1)       # L = 8192: supported
    assert L.workspace_bytes(ok) > 2 * 8192 * 8192 * 16


def test_bench_roofline_traffic_uses_committed_pmc():
    """bench.py's roofline.traffic comes from the committed PMC summaries: every phase's
    anchor kernel must be present in them, or the bench line silently reports null
    (the B^H kernel's rename once did exactly that)."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("sbce_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    with open(os.path.join(ROOT, "profiles", "pmc_cfg1_latest.json")) as f:
        pmc1 = json.load(f)
    assert pmc1["config"] == "cfg1" and pmc1["trials"] == 1000
    m = bench.phase_traffic(pmc1, bench.MSTEP_KERNELS, bench.MSTEP_ANCHORS)
    e = bench.phase_traffic(pmc1, bench.ESTEP_KERNELS, bench.ESTEP_KERNELS)
    assert m is not None and e is not None
    # above the algorithmic floor of one 1000-trial M-step
    assert m > bench.mstep_bytes_per_trial_iter(4, 4, 64, 16, 256) * 1000
    with open(os.path.join(ROOT, "profiles", "pmc_cfg2_latest.json")) as f:
        pmc2 = json.load(f)
    assert bench.phase_traffic(pmc2, bench.MSTEP_KERNELS_LARGE, bench.MSTEP_ANCHORS) is not None
    assert bench.phase_traffic({}, bench.MSTEP_KERNELS, bench.MSTEP_ANCHORS) is None


def test_committed_roofline_fractions_are_physical():
    """the roofline fraction must follow from the work the kernel executes.  From
    the committed round profiles alone (profiles/r03): the dominant kernel's executed flops
    (bench.py's count) over its rocprofv3 average duration is at most the FP64 peak and at most
    the measured FP64 MFMA pipe rate (with 5 % timing slack), and the bench line's own frac
    agrees with that recomputation."""
    import csv
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("sbce_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    d = os.path.join(ROOT, "profiles", "r03")
    line = [l for l in open(os.path.join(d, "bench_cfg1.log")) if l.startswith("{")][-1]
    roof = json.loads(line)["roofline"]
    assert roof["kernel"] == "rbuild_herm_kernel"
    flops = bench.rbuild_flops_per_trial_iter(4, 64, 16, 256) * 1000
    assert abs(roof["flops_per_launch"] / flops - 1) < 1e-12
    with open(os.path.join(d, "kernel_stats_cfg1.csv")) as f:
        rows = [r for r in csv.DictReader(f) if "rbuild_herm_kernel" in r["Name"]]
    # the whole-batch launches (bench.py times the build alone at the full batch; its timed
    # region may run the batch as stream sub-batches: smaller grids, separate rows)
    row = max(rows, key=lambda r: float(r.get("Grid") or 0))
    tflops = flops / (float(row["AverageNs"]) * 1e-9) / 1e12
    assert tflops / bench.FP64_PEAK_TFLOPS <= 1.0
    assert tflops / roof["measured_pipe_tflops"] <= 1.05
    assert roof["frac"] <= 1.0 and roof["frac_of_measured_pipe"] <= 1.05
    # the bench's live HIP-event timing and the profiler's average agree
    assert abs(roof["ms"] / (float(row["AverageNs"]) * 1e-6) - 1) < 0.05
    assert roof["traffic_ratio"] >= 1.0 - 0.05


def test_library_shares_torchs_hip_runtime(sbce):
    """libsbce.so must resolve libamdhip64.so.7 to the HIP runtime torch already loaded (torch's
    ROCm wheel bundles its own); loading it first would bring in a second runtime, whose launches
    then fail with hipErrorNoDevice.  _lib.load() imports torch before dlopen."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import importlib; "
            "m = importlib.import_module(%r); m._lib.load(); "
            "maps = open('/proc/self/maps').read(); "
            "print(len({l.split()[-1] for l in maps.splitlines() if 'libamdhip64' in l}))"
            % (ROOT, "semi-blind-channel-estimation-for-mimo-ris-communication-system-using-em-algo_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip() == "1", out.stdout
