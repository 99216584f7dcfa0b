"""EngineContext: owns one CKKS Engine and its key set (reference: engine_context.py:9-85).

Same constructor (three desilofhe Engine signatures selected by ``signature``) and the same
keys: secret, public, relinearisation, conjugation, rotation, optional fixed-rotation keys and
the two bootstrap keys.  The Engine is the MI355X HIP engine (fhe.Engine).
"""
from __future__ import annotations

from .fhe import Engine


class EngineContext:
    def __init__(self, signature: int, *, max_level: int = 30, mode: str = "cpu",
                 use_bootstrap: bool = True, use_multiparty: bool = False,
                 thread_count: int = 0, device_id: int = 0, fixed_rotation: bool = False,
                 delta_list: list | None = None, log_coeff_count: int = 0,
                 special_prime_count: int = 0, **engine_overrides) -> None:
        common = dict(mode=mode, use_multiparty=use_multiparty, thread_count=thread_count,
                      device_id=device_id, **engine_overrides)
        if signature == 1:
            self.engine = Engine(use_bootstrap=use_bootstrap, **common)
        elif signature == 2:
            self.engine = Engine(max_level=max_level, **common)
        elif signature == 3:
            self.engine = Engine(log_coeff_count=log_coeff_count,
                                 special_prime_count=special_prime_count, **common)
        else:
            raise ValueError(f"Unsupported signature: {signature}")

        eng = self.engine
        self.secret_key = eng.create_secret_key()
        self.public_key = eng.create_public_key(self.secret_key)
        self.relinearization_key = eng.create_relinearization_key(self.secret_key)
        self.conjugation_key = eng.create_conjugation_key(self.secret_key)
        self.rotation_key = eng.create_rotation_key(self.secret_key)
        self.fixed_rotation_key_list = []
        if fixed_rotation and delta_list is not None:
            self.fixed_rotation_key_list = [eng.create_fixed_rotation_key(self.secret_key, d)
                                            for d in delta_list]
        self.small_bootstrap_key = eng.create_small_bootstrap_key(self.secret_key)
        self.bootstrap_key = eng.create_bootstrap_key(self.secret_key)

    def __repr__(self) -> str:  # pragma: no cover
        e = self.engine
        return (f"<EngineContext N=2^{e.log_coeff_count} L={e.max_level} "
                f"slots={e.slot_count} backend={e._lib.backend}>")

    def encrypt(self, data):
        return self.engine.encrypt(data, self.public_key)

    def decrypt(self, ct):
        return self.engine.decrypt(ct, self.secret_key)
