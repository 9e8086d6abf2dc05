"""The host code of the path that runs without a device, under sanitizers
("ASan/TSan on the CPU reference build"): tests/native/
san_main.cpp built with -fsanitize=address,undefined (every report fatal) and
with -fsanitize=thread, linking the CPU oracle (oracle/orb_oracle.cpp), the
product's text-vocabulary parser and BoW assembly (csrc/vocab.cpp) and its
batch gather (csrc/host_gather.h) from their sources.  The ASan/UBSan driver
extracts the configs' frame shapes and runs every matcher entry point of the
oracle, parses well-formed, truncated and malformed vocabulary files and
gathers 64 frames on 4 threads; the TSan driver extracts on 4 threads with a
handle each (bench.py's CPU-baseline model) and gathers 128 frames on 8.
tools/sanitize_cpu_suite.sh also runs the whole CPU suite against an ASan
build of the oracle."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
NATIVE = ROOT / "tests" / "native"
sys.path.insert(0, str(ROOT / "tests"))


@pytest.fixture(scope="module")
def drivers():
    if not shutil.which("g++"):
        pytest.skip("no g++")
    r = subprocess.run(["make", "-s", "-C", str(NATIVE), "san"], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        if "cannot find -lasan" in r.stderr or "libtsan" in r.stderr:
            pytest.skip("sanitizer runtimes absent")
        raise AssertionError(r.stderr[-3000:])
    return NATIVE / "bin" / "san_driver", NATIVE / "bin" / "tsan_driver"


@pytest.fixture(scope="module")
def vocab_dir(tmp_path_factory):
    from vocab_ref import save_text

    from orb_slam3_vio_fixes_amd import synth
    d = tmp_path_factory.mktemp("voc")
    save_text(d / "k4_l3.txt", synth.vocabulary(4, 3, seed=3), 4)
    save_text(d / "k10_l2_no_newline.txt", synth.vocabulary(10, 2, seed=4), 10, trailing_newline=False)
    (d / "truncated.txt").write_text("10 6 0 0\n0 0 1 2 3")
    (d / "bad_header.txt").write_text("garbage\n")
    (d / "empty.txt").write_text("")
    (d / "negative_parent.txt").write_text("2 1 0 0\n-5 1 " + " ".join(["7"] * 32) + " 0.5\n")
    (d / "huge_k.txt").write_text("99999999 99 0 0\n")
    return d


def test_asan_ubsan_driver(drivers, vocab_dir):
    r = subprocess.run([str(drivers[0]), "all", str(vocab_dir)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1",
                            "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "vocabulary files 7" in r.stdout and "gather 64 frames on 4 threads" in r.stdout


def test_tsan_driver(drivers, vocab_dir):
    r = subprocess.run([str(drivers[1]), "threads", str(vocab_dir)], capture_output=True, text=True, timeout=300,
                       env={"TSAN_OPTIONS": "halt_on_error=1", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr
    assert "gather 128 frames on 8 threads" in r.stdout
