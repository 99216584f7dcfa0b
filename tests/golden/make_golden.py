#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE's own Python services (test infrastructure).

desilofhe (the reference's closed CKKS engine) is absent and unfetchable, so the reference's
services (/root/reference: xor_service.py, new.py, sbox/sbox_service.py, shiftrows_service.py,
shift_mix_zeta.py, mixcolumns_service.py) are imported here over an exact-arithmetic stand-in
of desilofhe.Engine: slot vectors are complex128 numpy arrays, every multiplication lowers the
level by one, make_power_basis(ct, d) returns ct^k at level L - ceil(log2 k), rotate is
np.roll (test/test_engine_rot.py:38-40), relinearize of a 2-polynomial ciphertext raises
"should have 3 polynomials" (the string matched at xor_service.py:116) and bootstrap is the
identity that restores the top level.  Every engine call is appended to a trace.

The reference sources are read in place from /root/reference and never copied; this script
only runs in the build container.  Output (committed):
  golden.npz   decoded outputs + their inputs (XOR, ARK, SubBytes, ShiftRows, MixRow, GF x2/x3
               and the GF coefficient vectors the reference's generator makes)
  traces.json  op-count traces of each service call (incl. GF mul2/mul3, AESFHETransformer)
Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import math
import sys
import types
from collections import Counter
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
SLOTS = 32768
MAX_LEVEL = 30


# ------------------------------------------------------------------------------------------
# exact-arithmetic stand-in of desilofhe
class Ciphertext:
    def __init__(self, v, level):
        self.v, self.level = v, level


class Plaintext:
    def __init__(self, v):
        self.v = v


class _Key:
    pass


class Engine:
    trace: list = []

    def __init__(self, *a, **kw):
        self.slot_count = SLOTS

    def _t(self, name, lvl=None):
        Engine.trace.append(name)

    def _pad(self, data):
        v = np.zeros(SLOTS, dtype=np.complex128)
        d = np.asarray(data, dtype=np.complex128).ravel()
        v[:d.size] = d
        return v

    def create_secret_key(self): return _Key()
    def create_public_key(self, sk): return _Key()
    def create_relinearization_key(self, sk): return _Key()
    def create_conjugation_key(self, sk): return _Key()
    def create_rotation_key(self, sk): return _Key()
    def create_fixed_rotation_key(self, sk, d): return _Key()
    def create_small_bootstrap_key(self, sk): return _Key()
    def create_bootstrap_key(self, sk): return _Key()

    def encode(self, vec):
        self._t("encode")
        return Plaintext(self._pad(vec))

    def encrypt(self, data, key):
        self._t("encrypt")
        return Ciphertext(self._pad(data), MAX_LEVEL)

    def decrypt(self, ct, key):
        self._t("decrypt")
        return ct.v.copy()

    def add(self, a, b):
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            self._t("add_ct_ct")
            return Ciphertext(a.v + b.v, min(a.level, b.level))
        ct, pt = (a, b) if isinstance(a, Ciphertext) else (b, a)
        self._t("add_ct_pt")
        return Ciphertext(ct.v + pt.v, ct.level)

    def multiply(self, a, b, rlk=None):
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            self._t("mul_ct_ct")
            return Ciphertext(a.v * b.v, min(a.level, b.level) - 1)
        ct, o = (a, b) if isinstance(a, Ciphertext) else (b, a)
        if isinstance(o, Plaintext):
            self._t("mul_ct_pt")
            return Ciphertext(ct.v * o.v, ct.level - 1)
        self._t("mul_ct_scalar")
        return Ciphertext(ct.v * complex(o), ct.level - 1)

    def make_power_basis(self, ct, d, rlk):
        self._t(f"power_basis_{d}")
        return [Ciphertext(ct.v ** k, ct.level - math.ceil(math.log2(k)) if k > 1 else ct.level)
                for k in range(1, d + 1)]

    def conjugate(self, ct, key):
        self._t("conjugate")
        return Ciphertext(np.conj(ct.v), ct.level)

    def rotate(self, ct, key, k):
        self._t("rotate")
        return Ciphertext(np.roll(ct.v, k), ct.level)

    def relinearize(self, ct, rlk):
        self._t("relinearize")
        raise RuntimeError("Input ciphertext should have 3 polynomials")

    def bootstrap(self, ct, *keys):
        self._t("bootstrap")
        return Ciphertext(ct.v.copy(), MAX_LEVEL)


def install():
    mod = types.ModuleType("desilofhe")
    mod.Engine, mod.Ciphertext, mod.Plaintext = Engine, Ciphertext, Plaintext
    sys.modules["desilofhe"] = mod
    sys.dont_write_bytecode = True
    pkg = types.ModuleType("aes_xor_fhe")
    pkg.__path__ = [str(REF)]
    sys.modules["aes_xor_fhe"] = pkg
    sys.path.insert(0, str(REF))        # bare imports (xor_service.py:13, new.py:4-5)


def counts(fn):
    Engine.trace = []
    out = fn()
    return out, dict(Counter(Engine.trace))


def main():
    install()
    import aes_xor_fhe.xor_service as xs
    import aes_xor_fhe.new as new
    import aes_xor_fhe.shiftrows_service as srs
    import aes_xor_fhe.shift_mix_zeta as smz
    from aes_xor_fhe.sbox import sbox_service as sbs
    import aes_xor_fhe.engine_context as ec

    # numpy-2 compatibility of the reference's ZetaEncoder: cast to int64
    def to_zeta(arr, modulus=16):
        a = np.asarray(arr).astype(np.int64)
        return np.exp(-2j * np.pi * (a % modulus) / modulus)
    xs.ZetaEncoder.to_zeta = staticmethod(to_zeta)

    g, traces = {}, {}
    cfg = xs.XORConfig(coeffs_path=REF / "generator" / "coeffs" / "xor_mono_coeffs.json")
    ew = xs.EngineWrapper(cfg)
    svc = xs.XORService(ew, xs.CoefficientCache(cfg.coeffs_path))

    # 4-bit XOR, 32768 random nibble pairs (test/test_xor_service.py:38-43, seed 0)
    rng = np.random.default_rng(0)
    a = rng.integers(0, 16, size=SLOTS, dtype=np.uint8)
    b = rng.integers(0, 16, size=SLOTS, dtype=np.uint8)
    out, traces["xor"] = counts(lambda: svc.xor(a, b))
    g["xor_a"], g["xor_b"], g["xor_out"] = a, b, out

    # every nibble pair in one SIMD ciphertext (test_nibble_xor_bruteforce semantics)
    pa, pb = np.repeat(np.arange(16, dtype=np.uint8), 16), np.tile(np.arange(16, dtype=np.uint8), 16)
    g["xor_all_out"] = svc.xor(pa, pb)[:256]

    # nibble-domain AddRoundKey full_round (new.py main: seed 1, 32768 bytes)
    rng = np.random.default_rng(1)
    st = rng.integers(0, 256, size=SLOTS, dtype=np.uint8)
    ky = rng.integers(0, 256, size=SLOTS, dtype=np.uint8)
    rnd = new.AESFHERound(ew, svc)
    out, traces["full_round"] = counts(lambda: rnd.full_round(st, ky, recombine=True))
    g["ark_state"], g["ark_key"], g["ark_out"] = st, ky, out
    # test_all_process.py:12-17 seeds (legacy RandomState)
    np.random.seed(25073101)
    s16 = np.random.randint(0, 256, 16, dtype=np.uint8)
    np.random.seed(25073102)
    k16 = np.random.randint(0, 256, 16, dtype=np.uint8)
    g["ark16_state"], g["ark16_key"] = s16, k16
    g["ark16_out"] = rnd.full_round(s16, k16, recombine=True)

    # SubBytes: 0..255 tiled over all slots (test/test_sbox_service.py:55-65)
    ctx = ec.EngineContext(signature=2, max_level=22, mode="parallel", thread_count=8)
    sb = sbs.SBoxService(ctx, hi_path=REF / "sbox/coeffs/sbox_hi_coeffs.json",
                         lo_path=REF / "sbox/coeffs/sbox_lo_coeffs.json")
    from aes_xor_fhe.utils import zeta_decode, zeta_encode
    plain = np.tile(np.arange(256, dtype=np.uint8), SLOTS // 256)
    enc = ctx.engine.encrypt(zeta_encode(plain, modulus=256), ctx.public_key)
    out, traces["sub_bytes_array"] = counts(lambda: sb.sub_bytes_array(enc))
    g["sbox_in"] = plain
    g["sbox_out"] = zeta_decode(ctx.engine.decrypt(out, ctx.secret_key), modulus=256)
    g["sbox_level_drop"] = np.array([MAX_LEVEL - out.level])

    # ShiftRows on contiguous 16-slot blocks (shiftrows_service.py:33-51): reference values
    sr = srs.AESFHEShiftRows(ew, svc)
    state = np.arange(16, dtype=np.int64)
    ct = ew.encrypt(np.asarray(state, dtype=np.float64))
    out, traces["shift_rows"] = counts(lambda: sr.shift_rows(ct))
    g["shiftrows_in"] = state
    g["shiftrows_out"] = np.real(ew.decrypt(out))[:16]
    # InvShiftRows (shiftrows_service.py:53-69) on the same state
    out, traces["inverse_shift_rows"] = counts(lambda: sr.inverse_shift_rows(ct))
    g["inv_shiftrows_out"] = np.real(ew.decrypt(out))[:16]

    # MixRow merged ShiftRows+MixColumns (shift_mix_zeta.py:14-69): op trace only
    mr = smz.MixRow(svc, ew)
    st4 = np.arange(16).reshape(4, 4) % 16
    out, traces["mixrow_merged_shift_mix"] = counts(lambda: mr.merged_shift_mix_fhe(st4))
    g["mixrow_abs_max"] = np.array([np.abs(ew.decrypt(out)).max()])

    # MixRow inverse (shift_mix_zeta.py:71-122): op trace and the values its final decrypt
    # decodes.  Its last line reshapes the whole slot vector into 4 x 4 (shift_mix_zeta.py:121)
    # and raises for any slot count above 16; the trace holds every engine call before that, the
    # 16 decoded values are taken from that final decrypt.
    from aes_xor_fhe.utils import zeta_decode as zd16
    inv_in = np.arange(16, dtype=np.float64) % 16
    ct_inv = ew.encrypt(zeta_encode(inv_in))
    last = {}
    orig_decrypt = Engine.decrypt

    def spy(self, ct, key):
        v = orig_decrypt(self, ct, key)
        last["v"] = v
        return v
    Engine.decrypt = spy
    Engine.trace = []
    try:
        mr.merged_inv_mixshift_fhe_from_ct(ct_inv)
        raised = ""
    except ValueError as ex:
        raised = str(ex)
    finally:
        Engine.decrypt = orig_decrypt
    traces["mixrow_merged_inv_mixshift"] = dict(Counter(Engine.trace))
    g["mixrow_inv_in"] = inv_in
    g["mixrow_inv_out"] = np.round(zd16(last["v"])).astype(np.int64)[:16].reshape(4, 4)
    g["mixrow_inv_reference_raises"] = np.array([bool(raised)])

    # GF(2^8) x2 / x3 (gf_service.py:55-78).  The coefficient files it loads are absent from the
    # reference tree; they are produced by the reference's own generator
    # (generator/generate_gf2_gf3_coeffs.py:47-70, main()) redirected into a temp dir, never
    # into /root/reference.
    import importlib
    import tempfile
    tmp = Path(tempfile.mkdtemp(prefix="aesfhe_gf_"))
    gen = importlib.import_module("aes_xor_fhe.generator.generate_gf2_gf3_coeffs")
    (tmp / "generator").mkdir()
    gen.__file__ = str(tmp / "generator" / "generate_gf2_gf3_coeffs.py")
    gen.main()
    import aes_xor_fhe.gf_service as gfs
    gfs.__file__ = str(tmp / "gf_service.py")      # base = tmp / "generator/coeffs"
    for k in ("gf2_hi", "gf2_lo", "gf3_hi", "gf3_lo"):
        g[f"{k}_coeffs"] = gfs._load_coeffs(tmp / "generator" / "coeffs" / f"{k}_coeffs.json")
    gf = gfs.GFService(ew, svc)
    gplain = np.tile(np.arange(256, dtype=np.uint8), SLOTS // 256)
    gct = ew.encrypt(zeta_encode(gplain, modulus=256))
    g["gf_in"] = gplain
    for name, fn in (("gf2", gf.mul2), ("gf3", gf.mul3)):
        (hi, lo), traces[f"gf_{name[2]}_mul"] = counts(lambda: fn(gct))
        g[f"{name}_hi_out"] = zeta_decode(ew.decrypt(hi), modulus=256)
        g[f"{name}_lo_out"] = zeta_decode(ew.decrypt(lo), modulus=256)
        g[f"{name}_level_drop"] = np.array([MAX_LEVEL - hi.level])

    # AESFHETransformer.merged_shift_mix (mixcolumns_service.py:21-83): op trace; its decoded
    # output diverges (8-bit zeta values through the 4-bit XOR LUT), so only finiteness is kept
    import aes_xor_fhe.mixcolumns_service as mcs
    tr = mcs.AESFHETransformer(ew, svc, gf)
    out, traces["transformer_merged_shift_mix"] = counts(
        lambda: tr.merged_shift_mix(np.arange(16, dtype=np.uint8)))
    g["transformer_out_finite"] = np.array([bool(np.all(np.isfinite(ew.decrypt(out))))])

    np.savez_compressed(OUT / "golden.npz", **g)
    (OUT / "traces.json").write_text(json.dumps(traces, indent=1, sort_keys=True))
    print("wrote", OUT / "golden.npz", OUT / "traces.json")
    for k, v in traces.items():
        print(k, v)


if __name__ == "__main__":
    main()
