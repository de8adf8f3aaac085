"""ASan + UBSan over the host C / C++ (SURVEY §5 "Race detection / sanitizers"): `make -C oracle
sanitize` builds the oracle, the ABI's host half (csrc/dpg_host.c), the workload generator
(csrc/dpg_synth.c) and the symbolic Cholesky (csrc/dpg_chol_sym.cpp) with
-fsanitize=address,undefined -fno-sanitize-recover=all and runs tools/sanitize_check.cpp through
them (scans -> clouds -> ICP -> GN -> symbolic analysis, full and incremental -> DPG change
detection); any report fails the run."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "sanitize check ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
