"""ctypes binding of the C ABI declared in include/aesfhe.h.

The same binding drives either implementation of the ABI:
  * the product library ``libaesfhe.so`` (HIP, gfx950) -- loaded by :func:`load_product`;
  * the CPU oracle ``oracle/_build/liboracle_ckks.so`` -- loaded only by tests/ and by
    bench.py's cpu_baseline leg, which pass the handle to ``Engine(_lib=...)`` explicitly.

The product loader never falls back to anything: if the HIP extension is missing or cannot be
loaded it raises, so a GPU run can never silently use a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
PRODUCT_LIB = _HERE.parent / "build" / "libaesfhe.so"

c_ct_p = C.c_void_p
c_key_p = C.c_void_p
c_pt_p = C.c_void_p
c_eng_p = C.c_void_p


class Params(C.Structure):
    _fields_ = [
        ("log_n", C.c_int32),
        ("max_level", C.c_int32),
        ("special_primes", C.c_int32),
        ("scale_bits", C.c_int32),
        ("base_bits", C.c_int32),
        ("special_bits", C.c_int32),
        ("device", C.c_int32),
        ("threads", C.c_int32),
        ("seed", C.c_uint64),
        ("primes", C.POINTER(C.c_uint64)),
        ("seed_ext", C.c_uint64 * 3),
        ("digit_primes", C.c_int32),
    ]


# (name, restype, argtypes) for every symbol of include/aesfhe.h
_P = C.POINTER
ABI_VERSION = 5  # include/aesfhe.h AESFHE_ABI_VERSION

SIGNATURES = [
    ("aesfhe_last_error", C.c_char_p, []),
    ("aesfhe_backend_name", C.c_char_p, []),
    ("aesfhe_abi_version", C.c_int32, []),
    ("aesfhe_engine_create", C.c_int, [_P(Params), _P(c_eng_p)]),
    ("aesfhe_engine_destroy", None, [c_eng_p]),
    ("aesfhe_engine_dims", C.c_int, [c_eng_p, _P(C.c_int32)]),
    ("aesfhe_engine_primes", C.c_int, [c_eng_p, _P(C.c_uint64)]),
    ("aesfhe_engine_scales", C.c_int, [c_eng_p, _P(C.c_double)]),
    ("aesfhe_engine_mul_scale", C.c_double, [c_eng_p, C.c_int32]),
    ("aesfhe_engine_sync", C.c_int, [c_eng_p]),
    ("aesfhe_engine_profile", C.c_int, [c_eng_p, C.c_int32]),
    ("aesfhe_engine_profile_read", C.c_int,
     [c_eng_p, C.c_char_p, _P(C.c_int64), _P(C.c_double), _P(C.c_double)]),
    ("aesfhe_engine_profile_kernels", C.c_int, [c_eng_p, C.c_char_p, C.c_int64, _P(C.c_int64)]),
    ("aesfhe_engine_device_bytes", C.c_int64, [c_eng_p]),
    ("aesfhe_engine_pool_stats", C.c_int, [c_eng_p, C.POINTER(C.c_int64)]),
    ("aesfhe_engine_pool_trim", C.c_int, [c_eng_p]),
    ("aesfhe_encode", C.c_int,
     [C.c_int32, _P(C.c_double), _P(C.c_double), C.c_int64, C.c_double, _P(C.c_int64)]),
    ("aesfhe_decode", C.c_int,
     [C.c_int32, _P(C.c_int64), C.c_double, _P(C.c_double), _P(C.c_double)]),
    ("aesfhe_chain", C.c_int, [_P(Params), _P(C.c_uint64), _P(C.c_double)]),
    ("aesfhe_key_secret", C.c_int, [c_eng_p, C.c_uint64, _P(c_key_p)]),
    ("aesfhe_key_public", C.c_int, [c_eng_p, c_key_p, _P(c_key_p)]),
    ("aesfhe_key_relin", C.c_int, [c_eng_p, c_key_p, _P(c_key_p)]),
    ("aesfhe_key_galois", C.c_int, [c_eng_p, c_key_p, C.c_uint64, _P(c_key_p)]),
    ("aesfhe_key_galois_hoisted", C.c_int, [c_eng_p, c_key_p, C.c_uint64, _P(c_key_p)]),
    ("aesfhe_galois_elt", C.c_uint64, [C.c_int32, C.c_int64, C.c_int32]),
    ("aesfhe_key_info", C.c_int, [c_key_p, _P(C.c_int32), _P(C.c_uint64)]),
    ("aesfhe_key_free", None, [c_key_p]),
    ("aesfhe_key_export", C.c_int,
     [c_eng_p, c_key_p, _P(C.c_int32), _P(C.c_uint64), _P(C.c_uint64), _P(C.c_int64), _P(C.c_uint64)]),
    ("aesfhe_key_import", C.c_int,
     [c_eng_p, C.c_int32, C.c_uint64, C.c_uint64, _P(C.c_uint64), C.c_int64, _P(c_key_p)]),
    ("aesfhe_key_trim", C.c_int, [c_eng_p, c_key_p, C.c_int32]),
    ("aesfhe_encrypt", C.c_int,
     [c_eng_p, c_key_p, _P(C.c_int64), C.c_int32, C.c_int32, C.c_uint64, _P(c_ct_p)]),
    ("aesfhe_decrypt", C.c_int, [c_eng_p, c_key_p, c_ct_p, _P(C.c_int64)]),
    ("aesfhe_encode_device", C.c_int,
     [c_eng_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_double, C.c_void_p]),
    ("aesfhe_decode_device", C.c_int, [c_eng_p, C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p]),
    ("aesfhe_encrypt_device", C.c_int,
     [c_eng_p, c_key_p, C.c_void_p, C.c_int32, C.c_int32, C.c_uint64, _P(c_ct_p)]),
    ("aesfhe_decrypt_device", C.c_int, [c_eng_p, c_key_p, c_ct_p, C.c_void_p]),
    ("aesfhe_ct_info", C.c_int, [c_ct_p, _P(C.c_int32)]),
    ("aesfhe_ct_export", C.c_int, [c_eng_p, c_ct_p, _P(C.c_uint64)]),
    ("aesfhe_ct_import", C.c_int,
     [c_eng_p, _P(C.c_uint64), C.c_int32, C.c_int32, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_ct_export_device", C.c_int, [c_eng_p, c_ct_p, C.c_int32, C.c_int32, C.c_void_p]),
    ("aesfhe_ct_import_device", C.c_int,
     [c_eng_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_ct_copy", C.c_int, [c_eng_p, c_ct_p, _P(c_ct_p)]),
    ("aesfhe_ct_slice", C.c_int, [c_eng_p, c_ct_p, C.c_int32, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_ct_concat", C.c_int, [c_eng_p, _P(c_ct_p), C.c_int32, _P(c_ct_p)]),
    ("aesfhe_ct_gather", C.c_int, [c_eng_p, c_ct_p, _P(C.c_int32), C.c_int32, _P(c_ct_p)]),
    ("aesfhe_ct_zero", C.c_int, [c_eng_p, C.c_int32, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_ct_free", None, [c_ct_p]),
    ("aesfhe_pt_create", C.c_int, [c_eng_p, _P(C.c_int64), C.c_int32, _P(c_pt_p)]),
    ("aesfhe_pt_create_ext", C.c_int, [c_eng_p, _P(C.c_int64), C.c_int32, _P(c_pt_p)]),
    ("aesfhe_pt_free", None, [c_pt_p]),
    ("aesfhe_add", C.c_int, [c_eng_p, c_ct_p, c_ct_p, _P(c_ct_p)]),
    ("aesfhe_sub", C.c_int, [c_eng_p, c_ct_p, c_ct_p, _P(c_ct_p)]),
    ("aesfhe_negate", C.c_int, [c_eng_p, c_ct_p, _P(c_ct_p)]),
    ("aesfhe_add_pt", C.c_int, [c_eng_p, c_ct_p, c_pt_p, _P(c_ct_p)]),
    ("aesfhe_add_const", C.c_int, [c_eng_p, c_ct_p, C.c_double, C.c_double, _P(c_ct_p)]),
    ("aesfhe_mul_pt", C.c_int, [c_eng_p, c_ct_p, c_pt_p, _P(c_ct_p)]),
    ("aesfhe_mul_const", C.c_int, [c_eng_p, c_ct_p, C.c_double, C.c_double, _P(c_ct_p)]),
    ("aesfhe_tensor", C.c_int, [c_eng_p, c_ct_p, c_ct_p, _P(c_ct_p)]),
    ("aesfhe_relinearize", C.c_int, [c_eng_p, c_ct_p, c_key_p, _P(c_ct_p)]),
    ("aesfhe_rescale", C.c_int, [c_eng_p, c_ct_p, _P(c_ct_p)]),
    ("aesfhe_mul", C.c_int, [c_eng_p, c_ct_p, c_ct_p, c_key_p, _P(c_ct_p)]),
    ("aesfhe_level_down", C.c_int, [c_eng_p, c_ct_p, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_galois", C.c_int, [c_eng_p, c_ct_p, c_key_p, _P(c_ct_p)]),
    ("aesfhe_mul_fma", C.c_int, [c_eng_p, c_ct_p, c_ct_p, c_key_p, C.c_int64, c_ct_p, C.c_double, C.c_double, _P(c_ct_p)]),
    ("aesfhe_rotate_hoisted", C.c_int, [c_eng_p, c_ct_p, _P(c_key_p), C.c_int32, _P(c_ct_p)]),
    ("aesfhe_power_basis", C.c_int, [c_eng_p, c_ct_p, C.c_int32, c_key_p, _P(c_ct_p)]),
    ("aesfhe_lincomb", C.c_int,
     [c_eng_p, _P(c_ct_p), C.c_int32, _P(C.c_double), _P(C.c_double), _P(c_ct_p)]),
    ("aesfhe_lincomb_many", C.c_int,
     [c_eng_p, _P(c_ct_p), C.c_int32, _P(C.c_double), _P(C.c_double), C.c_int32, _P(c_ct_p)]),
    ("aesfhe_dot", C.c_int, [c_eng_p, _P(c_ct_p), _P(c_ct_p), C.c_int32, c_key_p, _P(c_ct_p)]),
    ("aesfhe_dot_fma", C.c_int, [c_eng_p, _P(c_ct_p), _P(c_ct_p), C.c_int32, _P(c_ct_p), _P(C.c_double),
                                 C.c_int32, C.c_double, c_key_p, _P(c_ct_p)]),
    ("aesfhe_poly2", C.c_int,
     [c_eng_p, _P(c_ct_p), C.c_int32, _P(c_ct_p), C.c_int32, _P(C.c_double), _P(C.c_double),
      C.c_int32, c_key_p, _P(c_ct_p)]),
    ("aesfhe_poly2_int", C.c_int,
     [c_eng_p, _P(c_ct_p), C.c_int32, _P(c_ct_p), C.c_int32, _P(C.c_int32), C.c_int32,
      C.c_int32, c_key_p, _P(c_ct_p)]),
    ("aesfhe_poly2_int_rot", C.c_int,
     [c_eng_p, _P(c_ct_p), C.c_int32, _P(c_ct_p), C.c_int32, _P(C.c_int32), C.c_int32,
      C.c_int32, c_key_p, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_key_secret_sparse", C.c_int, [c_eng_p, C.c_uint64, C.c_int32, _P(c_key_p)]),
    ("aesfhe_key_switch", C.c_int, [c_eng_p, c_key_p, c_key_p, _P(c_key_p)]),
    ("aesfhe_mod_raise", C.c_int, [c_eng_p, c_ct_p, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_mul_i", C.c_int, [c_eng_p, c_ct_p, C.c_int32, _P(c_ct_p)]),
    ("aesfhe_dot_pt", C.c_int, [c_eng_p, _P(c_ct_p), _P(c_pt_p), C.c_int32, _P(c_ct_p)]),
    ("aesfhe_linear_bsgs", C.c_int,
     [c_eng_p, c_ct_p, C.c_int32, _P(c_key_p), C.c_int32, _P(c_key_p), _P(C.c_int32),
      _P(C.c_int32), _P(c_pt_p), _P(c_ct_p)]),
    ("aesfhe_ntt_host", C.c_int,
     [c_eng_p, _P(C.c_uint64), C.c_int32, _P(C.c_int32), C.c_int32]),
    ("aesfhe_bench_ntt", C.c_int,
     [c_eng_p, C.c_int32, C.c_int32, _P(C.c_double), _P(C.c_double)]),
]

SYMBOLS = [s[0] for s in SIGNATURES]

# error code -> exception message prefix (desilofhe raises RuntimeError with text; the
# reference matches "should have 3 polynomials" at xor_service.py:114-118)
ERRORS = {-1: "invalid argument", -2: "out of memory", -3: "device error",
          -4: "degree error", -5: "level error", -6: "unsupported"}


class Lib:
    """A loaded implementation of the aesfhe ABI."""

    def __init__(self, path: str | os.PathLike):
        self.path = str(path)
        self.cdll = C.CDLL(self.path, mode=C.RTLD_LOCAL)
        # the header revision first: a library built against an older header may lack newer
        # symbols (aesfhe_abi_version itself included), which must read as "rebuild it", not as
        # a ctypes "undefined symbol" from the binding loop
        stale = "?"
        try:
            ver = self.cdll.aesfhe_abi_version
            ver.restype, ver.argtypes = C.c_int, []
            stale = ver()
        except AttributeError:
            pass
        if stale != ABI_VERSION:
            raise RuntimeError(f"{self.path}: C ABI revision {stale}, this package needs "
                               f"{ABI_VERSION} (include/aesfhe.h AESFHE_ABI_VERSION): rebuild it")
        for name, res, args in SIGNATURES:
            try:
                fn = getattr(self.cdll, name)
            except AttributeError:
                raise RuntimeError(f"{self.path}: C ABI revision {ABI_VERSION} but symbol {name} is missing: "
                                   f"rebuild it") from None
            fn.restype = res
            fn.argtypes = args
            setattr(self, name[len("aesfhe_"):], fn)
        self.backend = self.backend_name().decode()

    def check(self, rc: int) -> None:
        if rc != 0:
            msg = self.last_error().decode(errors="replace")
            raise RuntimeError(f"[{self.backend}] {ERRORS.get(rc, 'error')}: {msg}")


_PRODUCT: Lib | None = None
PRODUCT_BACKEND = "hip-gfx950"


def load_product() -> Lib:
    """Load the HIP engine.  Raises if the extension has not been built -- there is no
    fallback implementation on the product path."""
    global _PRODUCT
    if _PRODUCT is None:
        # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (SONAME
        # libamdhip64.so.7) and loads it by file name, so if our library were loaded first the
        # process would end up with two HSA runtimes fighting over /dev/kfd.  Importing torch
        # first makes the dynamic loader resolve our DT_NEEDED libamdhip64.so.7 to that same
        # runtime (SONAME match), which is also what torch.distributed / RCCL use.
        try:
            import torch  # noqa: F401
        except Exception:  # torch absent: /opt/rocm's runtime is then the only one
            pass
        path = Path(os.environ.get("AESFHE_LIB", PRODUCT_LIB))
        if not path.exists():
            raise RuntimeError(
                f"aes-fhe HIP extension not found at {path}; build it with "
                f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        lib = Lib(path)
        # AESFHE_LIB selects another build of the product (A/B runs), never another backend: a
        # library that is not the gfx950 HIP engine (e.g. the CPU oracle) is refused here, so a
        # stray setting cannot turn a GPU test or the bench into the checker comparing itself
        if lib.backend != PRODUCT_BACKEND:
            raise RuntimeError(f"{path} is backend {lib.backend!r}, not the product ({PRODUCT_BACKEND!r})")
        _PRODUCT = lib
    return _PRODUCT
