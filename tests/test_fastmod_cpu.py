"""The double-multiply remainder and quotient of kh_device.h (mod_f64_32:
local_bin's h % p for tables below 2^30 bins, the reference's
`khash % _tablesizes[i]`, include/oxli/storage.hh:577; div_f64: the read of a
k-mer index in fixed-length batches) equal the integer operators over their
preconditions: the benchmark primes and edge sizes, every 2-bit k whose hashes
stay below 2^31 table sizes, and the quotient boundaries."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_fastmod_matches_integer_ops(tmp_path):
    exe = tmp_path / "fastmod_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "fastmod_check.cpp")],
                   check=True)
    out = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout
