"""Engine-call tracing with the categories of the golden stand-in trace
(tests/golden/make_golden.py), shared by the oracle and GPU service tests."""
from collections import Counter

from aes_xor_fhe.engine_context import EngineContext
from aes_xor_fhe.fhe import Ciphertext, Engine, Plaintext
from aes_xor_fhe.xor_service import EngineWrapper, XORConfig


class Tracing(Engine):
    """Counts engine calls with the categories of the golden stand-in trace."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.trace = Counter()

    def encode(self, vec, *a, **k):
        self.trace["encode"] += 1
        return super().encode(vec, *a, **k)

    def encrypt(self, data, key, level=None):
        self.trace["encrypt"] += 1
        return super().encrypt(data, key, level)

    def decrypt(self, ct, sk):
        self.trace["decrypt"] += 1
        return super().decrypt(ct, sk)

    def add(self, a, b):
        both = isinstance(a, Ciphertext) and isinstance(b, Ciphertext)
        self.trace["add_ct_ct" if both else "add_ct_pt"] += 1
        return super().add(a, b)

    def multiply(self, a, b, relinearization_key=None):
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            self.trace["mul_ct_ct"] += 1
        elif isinstance(a, Plaintext) or isinstance(b, Plaintext):
            self.trace["mul_ct_pt"] += 1
        else:
            self.trace["mul_ct_scalar"] += 1
        return super().multiply(a, b, relinearization_key)

    def make_power_basis(self, ct, degree, rlk):
        self.trace[f"power_basis_{degree}"] += 1
        return super().make_power_basis(ct, degree, rlk)

    def conjugate(self, ct, key):
        self.trace["conjugate"] += 1
        return super().conjugate(ct, key)

    def rotate(self, ct, key, delta=None):
        self.trace["rotate"] += 1
        return super().rotate(ct, key, delta)

    def relinearize(self, ct, rlk):
        self.trace["relinearize"] += 1
        return super().relinearize(ct, rlk)

    def bootstrap(self, ct, *keys):
        """One "bootstrap" entry, as in the reference's trace; the engine calls inside the
        refresh are not counted."""
        self.trace["bootstrap"] += 1
        saved = self.trace
        self.trace = Counter()
        try:
            return super().bootstrap(ct, *keys)
        finally:
            self.trace = saved


def make_wrap(lib, log_n=10, L=12, K=4, tracing=False, **kw):
    cls = Tracing if tracing else Engine
    # EngineContext builds the engine itself; inject the class through a tiny subclass
    import aes_xor_fhe.engine_context as ec
    orig = ec.Engine
    ec.Engine = cls
    try:
        ctx = EngineContext(signature=1, log_n=log_n, max_level=L, special_primes=K, seed=9, _lib=lib, **kw)
    finally:
        ec.Engine = orig
    return EngineWrapper(XORConfig(), ctx=ctx)
