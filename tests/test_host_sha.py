"""Host SHA-256 of the transcript (verkle-kzg_amd/csrc/host/sha256.hpp): the SHA-NI path equals
the portable rounds and the FIPS 180-2 known answers (transcript.rs:28-62 hashes through it)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_sha256_shani_matches_portable(tmp_path):
    exe = tmp_path / "sha256_check"
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(HERE, "cpp", "sha256_check.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
