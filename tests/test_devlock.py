"""The device lock's writer preference (qwen3-tts-jetson_amd/csrc/devlock.h WPLock): a single-slot
generate (exclusive hold) queued beside overlapping shared holds gets the device within a bound, and a shared hold
requested behind a queued writer is still admitted (the frame-callback / vocoder-worker dependency cannot deadlock).
CPU only: tests/cpp/test_devlock.cpp built with g++ against the header."""
import os
import subprocess

from q3t_testutil import REPO


def test_devlock_writer_bound_and_reader_yield(tmp_path):
    exe = str(tmp_path / "test_devlock")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(REPO, "qwen3-tts-jetson_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "test_devlock.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
