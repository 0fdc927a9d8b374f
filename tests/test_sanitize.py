"""ASan + UBSan over the host side of libpqgpu (format.cpp Thrift parser, host.cpp chunk planner):
tools/sanitize/host_fuzz plans every fixture and the reference's must-not-crash images
(chunk_reader_test / deltabp_decoder_test / fuzz_test / page_v1_test regressions) plus seeded
mutations of each (byte flips, 0x00/0xff/0x80 bytes, truncations, duplicated ranges), with and
without CRC validation. CPU only: plan-only batches, no kernel launch."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")
EXE = os.path.join(SAN, "build", "host_fuzz")


@pytest.fixture(scope="module")
def host_fuzz():
    objs = [os.path.join(ROOT, "parquet-go-1_amd", "build", n) for n in ("kernels.o", "bytearray.o")]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("library objects not built (make -C parquet-go-1_amd)")
    r = subprocess.run(["make", "-s", "-j4", "-C", SAN], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return EXE


def test_host_parser_sanitized(host_fuzz):
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.parquet")))
    files += sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "must_not_crash", "*.bin")))
    r = subprocess.run([host_fuzz, "-m", "40", "-s", "3"] + files, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"))
    assert r.returncode == 0 and "host_fuzz:" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]
