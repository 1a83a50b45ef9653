"""Sanitizer fuzzing of the code that reads untrusted bytes (race
detection / sanitizers; host side only -- GPU sanitizers are not available).

tests/fuzz/Makefile builds two libFuzzer targets with AddressSanitizer + UBSan:
  fuzz_containers  the product's host parsers (7z header walk, xz backward
                   index, LZMA2 chunk splitter, batch planner), from the
                   product sources;
  fuzz_lanes       the kernels' per-lane code built for the host (LZMA through
                   the generic and LDS-placement lanes, which must agree; LZMA2;
                   BCJ2; x86 BCJ; the RISC converters).
Seeds: the committed golden fixtures (tests/fuzz/seeds.py).  Each run is
bounded (a fixed run count) so the CPU suite stays a few minutes; any ASan /
UBSan report or a disagreement between the two LZMA lanes fails the test.
"""
import os
import subprocess
import sys

import pytest

import native

ROOT = native.ROOT
BUILD = os.path.join(ROOT, "tests", "fuzz", "build")


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    subprocess.run(["make", "-s", "-j8", "-f", "tests/fuzz/Makefile"], cwd=ROOT, check=True)
    d = tmp_path_factory.mktemp("fuzz")
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "fuzz", "seeds.py"), str(d)],
                   check=True)
    return d


@pytest.mark.parametrize("target,sub,max_len", [("fuzz_containers", "containers", 131072),
                                                ("fuzz_lanes", "lanes", 65536)])
def test_fuzz_target_clean(corpus, target, sub, max_len):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    work = corpus / (sub + "_work")
    work.mkdir(exist_ok=True)
    r = subprocess.run([os.path.join(BUILD, target), "-runs=12000", f"-max_len={max_len}",
                        "-seed=1", "-rss_limit_mb=4096", str(work), str(corpus / sub)],
                       cwd=str(corpus), env=env, capture_output=True, text=True, timeout=600)
    tail = r.stderr[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
    assert "Done 12000 runs" in r.stderr, tail
