"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

rnnlogic_amd/csrc/graph.cpp — the CSR / compact-view / edge-table builder
(rnnl_graph_create, ref src/data.py:39-106) and the rule-trie builder
(rnnl_rules_create, ref src/predictors.py:165-199) — is compiled with g++
-fsanitize=address,undefined next to tests/asan/graph_host_check.cpp, whose
host stand-ins for hipMalloc / hipMemcpy / hipFree keep the "device" arrays
in host memory so that the check reads them back: 60 random graphs (R up to
70: two relation words) and rule sets against a naive restatement, every
upload failing in turn (error code, nothing leaked), invalid inputs.
GPU sanitizers are not available on the MI355X pool; this covers the host
side of the boundary."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                    reason="needs g++ and the ROCm headers")
def test_graph_builders_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "graph_host_check")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(HERE, "asan", "graph_host_check.cpp"), os.path.join(REPO, "rnnlogic_amd", "csrc", "graph.cpp"),
           "-o", exe]
    out = subprocess.run(cmd, capture_output=True, text=True)
    assert out.returncode == 0, out.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert run.returncode == 0, (run.stdout + run.stderr)[-4000:]
    assert "0 live blocks" in run.stdout
    print(run.stdout.strip())
