"""Device-resident client path (include/aesfhe.h aesfhe_*_device): the codec
and encryption on device buffers must equal the host path word for word.

CPU (oracle, whose "device" is host memory): the facade's encrypt_device / decrypt_device and
the row-sliced AES client path round-trip.  GPU: the HIP kernels of codec_dev.h against the host
codec aesfhe_encode / aesfhe_decode (bit-identical coefficients and slots) at N = 2^14 / 2^16 /
2^17, and encrypt_device / decrypt_device against encrypt / decrypt residue for residue."""
import ctypes as C

import numpy as np
import pytest
import torch

from aes_xor_fhe import aes_tables as T
from aes_xor_fhe.fhe import Engine


def _slots(eng, rng, B, ns, cplx=True):
    v = rng.uniform(-1, 1, (B, ns))
    return v + 1j * rng.uniform(-1, 1, (B, ns)) if cplx else v


def test_oracle_client_path_roundtrip(oracle_lib):
    e = Engine(_lib=oracle_lib, log_n=10, max_level=4, special_primes=2, seed=3)
    sk = e.create_secret_key(1)
    pk = e.create_public_key(sk)
    v = _slots(e, np.random.default_rng(0), 3, e.slot_count - 5)
    c1 = e.encrypt_device(torch.from_numpy(v), pk)
    e2 = Engine(_lib=oracle_lib, log_n=10, max_level=4, special_primes=2, seed=3)
    sk2 = e2.create_secret_key(1)
    c2 = e2.encrypt(v, e2.create_public_key(sk2))
    assert np.array_equal(e.export_residues(c1), e2.export_residues(c2))  # same nonce, same words
    out = e.decrypt_device(c1, sk).numpy()
    assert np.array_equal(out, e.decrypt(c1, sk))
    np.testing.assert_allclose(out[:, :v.shape[1]], v, atol=1e-6)


def test_oracle_rows_client_path(oracle_lib):
    from aes_xor_fhe.aes_round_bits import AESRowRound
    e = Engine(_lib=oracle_lib, log_n=10, max_level=8, special_primes=3, seed=4)
    sk = e.create_secret_key(1)
    R = AESRowRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
    blocks = np.random.default_rng(1).integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
    st = R.encrypt_blocks_device(torch.from_numpy(blocks))
    rk = np.arange(16, dtype=np.uint8)
    out = R.decrypt_blocks_device(R.round(st, R.encrypt_round_key(rk)))
    assert np.array_equal(out.numpy(), T.aes_round(blocks, rk))


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [14, 16, 17])
def test_device_codec_bit_identical(product_lib, gpu_available, log_n):
    e = Engine(_lib=product_lib, log_n=log_n, max_level=3, special_primes=2, seed=5)
    n, N = e.slot_count, 1 << log_n
    rng = np.random.default_rng(log_n)
    dev = e.client_device
    for B, ns, cplx, scale in ((3, n, True, 2.0 ** 40), (2, n - 17, True, 2.0 ** 44), (1, n // 2, False, 2.0 ** 30)):
        v = _slots(e, rng, B, ns, cplx)
        re = torch.from_numpy(np.ascontiguousarray(v.real)).to(dev)
        im = torch.from_numpy(np.ascontiguousarray(v.imag)).to(dev) if cplx else None
        co = torch.empty((B, N), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        e._check(e._lib.encode_device(e._h, re.data_ptr(), im.data_ptr() if im is not None else None, B, ns, ns,
                                      scale, co.data_ptr()))
        got = co.cpu().numpy()
        for b in range(B):
            want = np.empty(N, np.int64)
            r_ = np.ascontiguousarray(v[b].real)
            i_ = np.ascontiguousarray(v[b].imag) if cplx else None
            e._check(e._lib.encode(log_n, r_.ctypes.data_as(C.POINTER(C.c_double)),
                                   i_.ctypes.data_as(C.POINTER(C.c_double)) if cplx else None, ns, scale,
                                   want.ctypes.data_as(C.POINTER(C.c_int64))))
            assert np.array_equal(got[b], want), f"encode differs (B={B}, ns={ns}, b={b})"
        # decode of those coefficients: slots bit-identical to the host decode
        ore = torch.empty((B, n), dtype=torch.float64, device=dev)
        oim = torch.empty((B, n), dtype=torch.float64, device=dev)
        e._check(e._lib.decode_device(e._h, co.data_ptr(), B, scale, ore.data_ptr(), oim.data_ptr()))
        e.synchronize()
        gr, gi = ore.cpu().numpy(), oim.cpu().numpy()
        for b in range(B):
            wr, wi = np.empty(n), np.empty(n)
            row = np.ascontiguousarray(got[b])
            e._check(e._lib.decode(log_n, row.ctypes.data_as(C.POINTER(C.c_int64)), scale,
                                   wr.ctypes.data_as(C.POINTER(C.c_double)), wi.ctypes.data_as(C.POINTER(C.c_double))))
            assert np.array_equal(gr[b], wr) and np.array_equal(gi[b], wi), "decode differs"
    # the overflow check matches the host codec's error
    big = torch.full((1, 4), 1e30, dtype=torch.float64, device=dev)
    co = torch.empty((1, N), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="overflows int64"):
        e._check(e._lib.encode_device(e._h, big.data_ptr(), None, 1, 4, 4, 2.0 ** 40, co.data_ptr()))


@pytest.mark.gpu
@pytest.mark.parametrize("log_n", [14, 16])
def test_device_encrypt_decrypt_equal_host(product_lib, gpu_available, log_n):
    kw = dict(log_n=log_n, max_level=5, special_primes=2, seed=8)
    a, b = Engine(_lib=product_lib, **kw), Engine(_lib=product_lib, **kw)
    ska, skb = a.create_secret_key(1), b.create_secret_key(1)
    pka, pkb = a.create_public_key(ska), b.create_public_key(skb)
    v = _slots(a, np.random.default_rng(2), 4, a.slot_count)
    ca = a.encrypt_device(torch.from_numpy(v), pka, level=4)
    cb = b._encrypt_host(v, pkb, 4)
    assert np.array_equal(a.export_residues(ca), b.export_residues(cb))
    for ct in (ca, a.multiply(ca, 0.5)):
        assert np.array_equal(a.decrypt_device(ct, ska).cpu().numpy(), a._decrypt_host(ct, ska))
    # the reference surface (Engine.encrypt / decrypt, engine_context.py:81-85) runs the device
    # codec on the HIP engine: the same words as the host codec, real and complex slots alike
    for x in (v, v.real, v[0], v[0, :100].real):
        c1, c2 = a.encrypt(x, pka, level=3), b._encrypt_host(x, pkb, 3)
        assert np.array_equal(a.export_residues(c1), b.export_residues(c2))
        assert np.array_equal(a.decrypt(c1, ska), a._decrypt_host(c1, ska))


@pytest.mark.gpu
def test_rows_client_path_gpu(product_lib, gpu_available):
    """blocks (device) -> pack / bit-slice / encode / encrypt on the GPU -> one AES round ->
    decrypt / decode / unpack on the GPU == FIPS-197, at N = 2^16."""
    from aes_xor_fhe.aes_round_bits import AESRowRound
    e = Engine(_lib=product_lib, log_n=16, max_level=10, special_primes=4, scale_bits=40, seed=6)
    sk = e.create_secret_key(1)
    R = AESRowRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
    blocks = np.random.default_rng(3).integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
    rk = np.random.default_rng(4).integers(0, 256, 16, dtype=np.uint8)
    st = R.encrypt_blocks_device(torch.from_numpy(blocks).to(e.client_device))
    out = R.decrypt_blocks_device(R.round(st, R.encrypt_round_key(rk)))
    assert out.device.type == "cuda"
    assert np.array_equal(out.cpu().numpy(), T.aes_round(blocks, rk))


@pytest.mark.gpu
def test_sliced_client_path_gpu(product_lib, gpu_available):
    """The bench's client_path leg in its exact form: AESSlicedRound (columns as batch elements,
    whole slabs of 4 sets, the last slab padded) packs / bit-slices / encodes / encrypts on the
    GPU, runs one round (ShiftRows folded into the S-box), decrypts / decodes / unpacks on the
    GPU == FIPS-197, at N = 2^16 with the bench's 12-prime digits over K = 10."""
    from aes_xor_fhe.aes_round_bits import AESSlicedRound
    e = Engine(_lib=product_lib, log_n=16, max_level=10, special_primes=10, digit_primes=12, scale_bits=40, seed=9)
    sk = e.create_secret_key(1)
    R = AESSlicedRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
    nb = 6  # two slabs, the second half padding
    blocks = np.random.default_rng(13).integers(0, 256, (nb, R.n_blk, 16), dtype=np.uint8)
    rk = np.random.default_rng(14).integers(0, 256, 16, dtype=np.uint8)
    st = R.encrypt_blocks_device(torch.from_numpy(blocks).to(e.client_device))
    assert st[0][0].batch == 8
    out = R.decrypt_blocks_device(R.round(st, R.encrypt_round_key(rk)), nb)
    assert out.device.type == "cuda" and tuple(out.shape) == (nb, R.n_blk, 16)
    assert np.array_equal(out.cpu().numpy(), T.aes_round(blocks, rk))
    # the host decryption of the same state agrees (device and host codecs are bit-identical)
    assert np.array_equal(R.decrypt_blocks(R.round(st, R.encrypt_round_key(rk)), nb), T.aes_round(blocks, rk))
