"""AddressSanitizer + UBSan runs of the host-side C/C++ (GPU sanitizers are not available on
this pool; host code only):
  * the CPU oracle (oracle/ckks_oracle.c) driven over the whole ABI by oracle/asan_check.c,
    engine destroyed before its objects (make -C oracle asan);
  * the HIP engine's host pieces (aes-fhe_amd/csrc/ckks_host.h: prime chain, roots, PRNG, codec)
    at every ring size, tests/native/host_asan.cpp; its device arena (arena.h); the linear_bsgs
    host planning (bsgs_plan.h).
A sanitizer report makes the program exit non-zero."""
import os
import subprocess

from conftest import ROOT

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", OMP_NUM_THREADS="2",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def test_oracle_asan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "asan"], check=True)
    r = subprocess.run([str(ROOT / "oracle" / "_build" / "asan_check")], env=ENV,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan_check ok" in r.stdout, r.stderr[-4000:]


def test_host_codec_asan(tmp_path):
    exe = tmp_path / "host_asan"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off",
                    "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-o", str(exe),
                    str(ROOT / "tests" / "native" / "host_asan.cpp")], check=True)
    r = subprocess.run([str(exe)], env=ENV, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "host_asan ok" in r.stdout, r.stderr[-4000:]


def test_oracle_chacha_kat(tmp_path):
    """The oracle's ChaCha20 stream against RFC 7539's block vector; the engine's
    host copy is checked in host_asan.cpp, and GPU-vs-oracle key equality (test_gpu_parity) ties
    the device kernels to both."""
    exe = tmp_path / "chacha_kat"
    subprocess.run(["gcc", "-std=gnu11", "-O1", "-fopenmp", "-fsanitize=address,undefined", "-o", str(exe),
                    str(ROOT / "tests" / "native" / "oracle_chacha_kat.c"), "-lm"], check=True)
    r = subprocess.run([str(exe)], env=ENV, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "oracle chacha ok" in r.stdout, (r.returncode, r.stderr[-2000:])


def test_device_arena_asan(tmp_path):
    """The engine's device arena (aes-fhe_amd/csrc/arena.h: best fit and first fit, neighbour merge, zero-copy
    split, trim, peak_live / fragmentation counters) over malloc under ASan + UBSan, against a
    shadow model (tests/native/arena_asan.cpp)."""
    exe = tmp_path / "arena_asan"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-o", str(exe), str(ROOT / "tests" / "native" / "arena_asan.cpp")], check=True)
    for mode in ([], ["first_fit"]):
        r = subprocess.run([str(exe)] + mode, env=ENV, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "arena_asan ok" in r.stdout, (mode, r.stdout[-2000:], r.stderr[-4000:])


def test_bsgs_plan_asan(tmp_path):
    """aesfhe_linear_bsgs's host planning (aes-fhe_amd/csrc/bsgs_plan.h: term validation, the
    giants' plaintext-pointer tables, the k-block walk order) under ASan + UBSan against a direct
    model (tests/native/bsgs_plan_asan.cpp)."""
    exe = tmp_path / "bsgs_plan_asan"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-o", str(exe), str(ROOT / "tests" / "native" / "bsgs_plan_asan.cpp")], check=True)
    r = subprocess.run([str(exe)], env=ENV, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "bsgs_plan_asan ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
