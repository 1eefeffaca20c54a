"""Host C code under AddressSanitizer + UBSan: the TFRecord
record walk and the protobuf Example parser of libjr read untrusted bytes
(mmap'd files), so the data-pipeline tests -- damaged and truncated files,
malformed / missing / duplicate features included -- run again against an
ASan+UBSan build of the same sources (csrc `make asan`: jr_host.cpp +
jr_error.cpp, no HIP), loaded through JR_HOST_LIB with libasan preloaded
into the (uninstrumented) interpreter.  Any sanitizer report fails the run."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "jama16-retina-replication_amd", "csrc")
LIB = os.path.join(ROOT, "jama16-retina-replication_amd", "jr", "libjr_host_asan.so")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_data_pipeline_under_asan():
    subprocess.run(["make", "-C", CSRC, "asan"], check=True, capture_output=True)
    libasan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, JR_HOST_LIB=LIB, LD_PRELOAD=libasan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_data_pipeline.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out
