"""CKKS bootstrapping over the engine primitives (Engine.bootstrap; the reference calls desilofhe's
at xor_service.py:120-129 and mixcolumns_service.py:72-75).

Pipeline for a ciphertext c at level 0 encrypting slots z (message m at the canonical scale D_0):

1. sparse-secret encapsulation: switch c to an ephemeral sparse ternary secret s' (hw nonzeros)
   at level 0, ModRaise to level L (now encrypts t = m + q_0 I with |I| <= K w.h.p.), switch back
   to the main secret s at level L;
2. CoeffToSlot: slots of the raised ciphertext are V u_t / D_L with u_k = t_k + i t_{k+n} and
   V_jk = xi^(5^j k) (verified against the codec); V = B_log(n) ... B_1 P (butterfly stages, P the
   bit reversal).  CtS applies (D_L / (2 q_0 Bnd)) B_1^-1 ... B_log(n)^-1 (merged into `groups`
   linear maps evaluated baby-step giant-step with aesfhe_dot_pt), giving the bit-reversed
   u_t / (2 q_0 Bnd);  x_re = w + conj(w), x_im = -i (w - conj(w)) hold t / (q_0 Bnd) in [-1, 1];
3. EvalMod: sin(2 pi Bnd x) via a Chebyshev approximation of cos(2 pi (Bnd x - 1/4) / 2^r) and r
   double-angle steps; sin(2 pi t/q_0) / (2 pi) = m / q_0 for |m| << q_0;
4. SlotToCoeff: (q_0 / (2 pi D_0)) B_log(n) ... B_1 applied to y_re + i y_im (the bit reversal
   cancels) returns the slots z at level L - depth.

Depth = 1 + 2 * groups + ceil(log2(deg + 1)) + 1 + r (16 with the defaults at any N).  The bit
mode (bootstrap_bits, StC first) spends groups levels before ModRaise and, with bits_opt,
groups + ceil(log2(deg + 1)) + r = 3 + 4 + 4 = 11 after it: c_in rides in the CtS diagonals and
the Chebyshev sum is evaluated depth-optimally (chebyshev_opt).
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np

from .fhe import Ciphertext, Engine


# ---- the encoding map in butterfly form --------------------------------------------------------
def _stage(n: int, N: int, length: int, inverse: bool) -> Dict[int, np.ndarray]:
    """Diagonal form {offset d: D_d} of one butterfly stage (block length `length`) of V or of its
    inverse: (S x)[p] = sum_d D_d[p] x[(p + d) mod n]."""
    h = length // 2
    M = 2 * N
    lenq = length << 2
    gap = M // lenq
    j = np.arange(h)
    w = np.exp(2j * np.pi * ((np.array([pow(5, int(x), lenq) for x in j]) * gap) % M) / M)
    p = np.arange(n)
    top = (p % length) < h
    jj = np.where(top, p % length, p % length - h)
    wp = w[jj]
    D0 = np.zeros(n, complex)
    Dp = np.zeros(n, complex)
    Dm = np.zeros(n, complex)
    if not inverse:  # top: x[p] + w x[p+h]; bottom: x[p-h] - w x[p]
        D0[top], Dp[top] = 1.0, wp[top]
        Dm[~top], D0[~top] = 1.0, -wp[~top]
    else:  # top: (x[p] + x[p+h]) / 2; bottom: conj(w) (x[p-h] - x[p]) / 2
        D0[top], Dp[top] = 0.5, 0.5
        Dm[~top], D0[~top] = np.conj(wp[~top]) / 2, -np.conj(wp[~top]) / 2
    out = {0: D0}
    for d, D in ((h % n, Dp), ((-h) % n, Dm)):  # h == -h (mod n) in the last stage: sum them
        out[d] = out.get(d, 0) + D
    return out


def _compose(A: Dict[int, np.ndarray], B: Dict[int, np.ndarray], n: int) -> Dict[int, np.ndarray]:
    """Diagonal form of A @ B: C_{a+b}[p] += A_a[p] B_b[p + a]."""
    C: Dict[int, np.ndarray] = {}
    for a, Da in A.items():
        for b, Db in B.items():
            d = (a + b) % n
            v = Da * np.roll(Db, -a)
            C[d] = C.get(d, 0) + v
    return {d: v for d, v in C.items() if np.any(np.abs(v) > 1e-14)}


def apply_diag(M: Dict[int, np.ndarray], x: np.ndarray) -> np.ndarray:
    return sum(D * np.roll(x, -d) for d, D in M.items())


def transform_groups(n: int, N: int, groups: int, inverse: bool) -> List[Dict[int, np.ndarray]]:
    """The log2(n) stages merged into `groups` maps, in application order.  Forward (StC):
    B_1 first ... B_log(n) last; inverse (CtS): B_log(n)^-1 first ... B_1^-1 last."""
    L = int(math.log2(n))
    lengths = [2 << s for s in range(L)]  # B_1 .. B_L block lengths 2 .. n
    order = list(reversed(lengths)) if inverse else lengths
    sizes = [len(a) for a in np.array_split(np.arange(L), groups)]
    out, i = [], 0
    for sz in sizes:
        M = None
        for length in order[i:i + sz]:  # later stages act after earlier ones: M = S @ M
            S = _stage(n, N, length, inverse)
            M = S if M is None else _compose(S, M, n)
        out.append(M)
        i += sz
    return out


def _bsgs_plan(offsets: List[int], n: int):
    """Offsets are k*u (k in a symmetric range); baby steps k1*u (0 <= k1 < g), giants g*k2*u."""
    nz = sorted(offsets)
    u = math.gcd(*[d for d in nz if d]) if any(nz) else 1
    u = math.gcd(u, n)
    ks = sorted({((d // u + n // (2 * u)) % (n // u)) - n // (2 * u) for d in nz})  # signed k
    span = max(ks) - min(ks) + 1
    g = 1 << max(0, math.ceil(math.log2(math.sqrt(span))))
    return u, ks, g


# ---- the bootstrapper --------------------------------------------------------------------------
class Bootstrapper:
    def __init__(self, engine: Engine, sk, rlk, cjk=None, *, hw: int = 32, K: float = 12.0,
                 r: int = 3, deg: int = 31, groups: int = 3, seed: int = 7,
                 bits_deg: int | None = None, bits_r: int | None = None, lazy: bool = True, baby_scale: int = 2,
                 bits_opt: bool = True, cts_groups: int | None = None, stc_baby_scale: float | None = None,
                 share: "Bootstrapper | None" = None):
        # cts_groups: CoeffToSlot's stages merged into this many maps (default `groups`, which
        # StC keeps): more groups = more levels, far fewer diagonals per map
        # share: a bootstrapper of the same engine and secret key whose key material this one
        # reuses -- the conjugation and sparse-secret keys, every rotation key of the same
        # rotation, and the SlotToCoeff plans (plaintext diagonals) when their parameters match.
        # The AES drivers run a 5-map and a 3-map CoeffToSlot bootstrapper side by side: their
        # StC maps are the same, and each held its own copy (config 5: 116 rotation keys of
        # 0.3 GB live at the N = 2^17 peak).
        cts_groups = groups if cts_groups is None else cts_groups
        self.groups, self.cts_groups = groups, cts_groups
        e = self.e = engine
        self.rlk = rlk
        if share is not None and share.e is not engine:
            raise ValueError("Bootstrapper(share=...) needs a bootstrapper of the same engine")
        # the secret key's identity: shared key material is only valid under the same key
        self._sk_seed = engine.key_seed(sk)
        if share is not None and share._sk_seed != self._sk_seed:
            raise ValueError("Bootstrapper(share=...) needs a bootstrapper of the same secret key")
        # a trimmed share's keys switch only at the SlotToCoeff levels: this bootstrapper's
        # CoeffToSlot (level L) would need the whole keys
        if share is not None and getattr(share, "_bits_only", False):
            raise ValueError("Bootstrapper(share=...) of a bootstrapper whose keys were trimmed "
                             "(trim_bootstrap_keys): build every sharing bootstrapper before trimming")
        self.cjk = cjk if cjk is not None else share.cjk if share is not None else e.create_conjugation_key(sk)
        self.N = 1 << e.log_coeff_count
        self.n = self.N // 2
        self.L = e.max_level
        self.r, self.deg, self.B = r, deg, K + 1.0
        # bits_opt: the bit mode folds c_in into the CoeffToSlot diagonals and evaluates EvalMod's
        # Chebyshev sum in depth ceil(log2(deg + 1)) (chebyshev_opt) -- two levels fewer (11
        # instead of 13), which is what lets ten AES rounds run on three refreshes
        self.bits_opt = bits_opt
        if bits_deg is None:
            bits_deg = 15 if bits_opt else 31
        if bits_r is None:
            bits_r = 4 if bits_opt else 3
        self.bits_deg, self.bits_r = bits_deg, bits_r
        # lazy: linear maps through aesfhe_linear_bsgs (baby rotations kept in Q u P, one ModDown
        # per giant + one for all giant key switches); baby steps are then cheap, so the BSGS
        # split takes baby_scale x more of them (fewer giants)
        self.lazy = lazy
        self.baby_scale = baby_scale if lazy else 1
        # SlotToCoeff runs at the bottom levels, where the K special primes are most of every
        # limb set: a giant's key switch costs about what a baby's Q u P ciphertext costs to
        # write and read back, so its split may take fewer babies (stc_baby_scale)
        self.stc_baby_scale = self.baby_scale if stc_baby_scale is None or not lazy else stc_baby_scale
        # sparse-secret encapsulation keys
        self._sparse_id = (hw, seed)
        if share is not None and share._sparse_id == self._sparse_id:
            self.to_sparse, self.from_sparse = share.to_sparse, share.from_sparse
        else:
            s_sparse = e.create_sparse_secret_key(hw, seed)
            # to_sparse only ever switches level-0 ciphertexts (_raise_to_slots): one digit kept
            self.to_sparse = e.trim_key(e.create_switching_key(sk, s_sparse), 0)
            self.from_sparse = e.create_switching_key(s_sparse, sk)
        q0 = float(e.primes[0])
        D = e.scales
        n, N = self.n, self.N
        # CtS: (D_L / (2 q0 Bnd)) * prod of inverse stages; StC: (q0 / (2 pi D_0)) * forward stages
        cts = transform_groups(n, N, cts_groups, inverse=True)
        stc = transform_groups(n, N, groups, inverse=False)
        # bit mode: c_in = D_L / (2 q0 Bnd) ~ 2^-15.7 spread over the CtS groups' diagonals
        # (c_in^(1/groups) each, plaintext integers ~2^30): the rounding it adds to t / q0 is
        # ~1e-7, and the bit mode's error enters squared
        self.B_bits = K + 1.0
        f_in = (D[self.L] / (2.0 * q0 * self.B_bits)) ** (1.0 / cts_groups)
        cts_bits = [{d: v * f_in for d, v in M.items()} for M in cts] if bits_opt else None
        # General mode: c_in folded into one group's diagonals would leave their plaintext integers
        # ~25 bits, and this mode's error is linear in it.  It is applied as its own constant multiply instead (one level): the
        # engine multiplies by exactly A / s (A = llround(c_in s)), and the bound is re-derived
        # from that value so that 2 pi Bnd x = 2 pi t / q0 holds exactly.
        s = e._lib.engine_mul_scale(e._h, self.L)
        self.c_in = round(D[self.L] / (2.0 * q0 * self.B) * s) / s
        self.B = D[self.L] / (2.0 * q0 * self.c_in)
        c_out = q0 / (2.0 * math.pi * D[0])
        stc_bits = [dict(M) for M in stc]
        stc[-1] = {d: v * c_out for d, v in stc[-1].items()}
        # bit mode: slots b + i b' -> coefficients (q0 / 4) (b, b') at level 0
        c_bits = q0 / (4.0 * D[0])
        stc_bits[-1] = {d: v * c_bits for d, v in stc_bits[-1].items()}
        self.cts = [self._prepare(M) for M in cts]
        # the StC plans depend on (groups, split, chain, the two output constants) only
        self._stc_id = (groups, self.stc_baby_scale, self.L, c_out, c_bits)
        if share is not None and share._stc_id == self._stc_id:
            self.stc, self.stc_bits = share.stc, share.stc_bits
            self._stc_bits_maps, self._stc_bits_scaled = share._stc_bits_maps, share._stc_bits_scaled
        else:
            self.stc = [self._prepare(M, self.stc_baby_scale) for M in stc]
            self.stc_bits = [self._prepare(M, self.stc_baby_scale) for M in stc_bits]
            self._stc_bits_maps = stc_bits  # for the scaled-input variants (bootstrap_bits in_scale)
            self._stc_bits_scaled: Dict[float, list] = {1.0: self.stc_bits}
        self.cts_bits = [self._prepare(M) for M in cts_bits] if bits_opt else self.cts
        # rotation keys: hoisted keys for the baby steps (one ModUp per group input), ordinary
        # keys for the giant steps
        babies, giants = set(), set()
        for plan in self.cts + self.stc:  # stc_bits has the offsets of stc
            u, g = plan["u"], plan["g"]
            babies.update((k1 * u) % n for k2, tl in plan["terms"].items() for k1, _ in tl if k1)
            giants.update((g * k2 * u) % n for k2 in plan["giants"] if (g * k2 * u) % n)
        hs, rs = (share.hrot, share.rot) if share is not None else ({}, {})
        self.hrot = {d: hs[d] if d in hs else e.create_hoisted_rotation_key(sk, -d) for d in sorted(babies)}
        self.rot = {d: rs[d] if d in rs else e.create_fixed_rotation_key(sk, -d) for d in sorted(giants)}
        # EvalMod: Chebyshev coefficients of cos(2 pi (Bnd x - 1/4) / 2^r) on [-1, 1], degree 31
        # and r = 3 (fit error 1.6e-13) in both modes.  A cheaper bit-mode fit (degree 15, r = 4:
        # same depth, 11 products instead of 14) leaves a sin error of 5.4e-5 that is the SAME
        # for every bit of a value, so it adds coherently through the S-box's Walsh polynomial
        # and the MixColumns products: full AES-128 failed at N = 2^10 with it (random noise of
        # 2e-4 does not), hence the bits_deg / bits_r knobs default to the general fit.
        # With bits_opt the bit mode uses degree 15 and r = 4 (depth 4 + 4, 7 + 4
        # relinearisations instead of 11 + 3 for degree 29 and r = 3), fitted where the bit mode
        # evaluates it (_bits_fit): the plain Chebyshev interpolant's error, 5.4e-5 at
        # t / q0 = +1/4 (I = 0, where all four double angles amplify it 4x), drops to ~2e-7.
        self.cheb = self._cheb_fit(deg, r, self.B)
        if bits_opt:
            self.cheb_bits = self._bits_fit(bits_deg, bits_r, self.B_bits, K)
        else:
            self.cheb_bits = self._cheb_fit(bits_deg, bits_r, self.B)
        self.depth = 1 + groups + cts_groups + math.ceil(math.log2(deg + 1)) + 1 + r
        self.bits_level = self.bits_output_level(self.L, cts_groups, bits_deg, bits_r, bits_opt)

    @staticmethod
    def bits_output_level(L: int, cts_groups: int = 3, bits_deg: int = 15, bits_r: int = 4,
                          bits_opt: bool = True) -> int:
        """bits_level of a Bootstrapper with these parameters (no keys made)."""
        cheb_depth = math.ceil(math.log2(bits_deg + 1)) + (0 if bits_opt else 1)
        return L - ((0 if bits_opt else 1) + cts_groups + cheb_depth + bits_r)

    @staticmethod
    def _bits_fit(deg: int, r: int, bnd: float, K: float, width: float = 1e-2,
                  weight: float = 1e3) -> np.ndarray:
        """Chebyshev coefficients of cos(2 pi (bnd x - 1/4) / 2^r) for the bit mode, by weighted
        least squares: 400 Chebyshev nodes of [-1, 1] (weight 1) plus the points the bit mode
        actually feeds it, x = (I +- 1/4 + d) / bnd for |I| <= K and |d| <= width (input bit errors
        up to 4 width), weighted by `weight` times the error gain of the r double angles there
        (prod |4 cos(2^k theta)|, 4^r at I = 0 and I = 2^(r-1), near 0 elsewhere)."""
        def f(x):
            return np.cos(2 * np.pi * (bnd * x - 0.25) / (1 << r))
        grid = np.cos(np.pi * (np.arange(400) + 0.5) / 400)
        dl = np.linspace(-width, width, 25)
        I = np.arange(-int(K), int(K) + 1)
        pts = np.concatenate([(i + s + dl) / bnd for i in I for s in (0.25, -0.25)])
        gain = np.ones_like(pts)
        c = f(pts)
        for _ in range(r):
            gain *= np.abs(4 * c)
            c = 2 * c * c - 1
        X = np.concatenate([grid, pts])
        w = np.concatenate([np.ones_like(grid), weight * gain / gain.max()])
        V = np.polynomial.chebyshev.chebvander(X, deg) * w[:, None]
        return np.linalg.lstsq(V, f(X) * w, rcond=None)[0]

    @staticmethod
    def _cheb_fit(deg: int, r: int, bnd: float) -> np.ndarray:
        kk = np.arange(deg + 1)
        xs = np.cos(np.pi * (kk + 0.5) / (deg + 1))
        f = np.cos(2 * np.pi * (bnd * xs - 0.25) / (1 << r))
        return np.polynomial.chebyshev.chebfit(xs, f, deg)

    def _prepare(self, M: Dict[int, np.ndarray], baby_scale: float | None = None):
        u, ks, g = _bsgs_plan(list(M), self.n)
        scale = self.baby_scale if baby_scale is None else baby_scale
        g = min(max(1, int(g * scale)), 1 << max(0, math.ceil(math.log2(max(ks) - min(ks) + 1))))
        giants = sorted({(k - (k % g)) // g for k in ks})
        terms = {}
        for k in ks:
            d = (k * u) % self.n
            k2 = (k - (k % g)) // g
            k1 = k - g * k2
            # sum_k2 rot( sum_k1 rot(D_k, -g k2 u) * rot(x, k1 u), g k2 u )
            terms.setdefault(k2, []).append((k1, self.e.encode(np.roll(M[d], g * k2 * u))))
        return {"u": u, "g": g, "giants": giants, "terms": terms}

    def _rot(self, ct: Ciphertext, d: int) -> Ciphertext:
        """x -> x[p + d] (d slots to the left)."""
        d %= self.n
        return ct if d == 0 else self.e.rotate(ct, self.rot[d])

    def linear(self, ct: Ciphertext, plan) -> Ciphertext:
        """sum_k D_k * rot(x, k u) as BSGS: the baby rotations of x in one hoisted call."""
        e, u, g = self.e, plan["u"], plan["g"]
        if self.lazy:
            terms = plan["terms"]
            ks = sorted({k1 for tl in terms.values() for k1, _ in tl})
            idx = {k1: i for i, k1 in enumerate(ks)}
            bkeys = [None if k1 == 0 else self.hrot[(k1 * u) % self.n] for k1 in ks]
            giants = sorted(terms)
            gkeys = [None if (g * k2 * u) % self.n == 0 else self.rot[(g * k2 * u) % self.n]
                     for k2 in giants]
            return e.linear_bsgs(ct, bkeys, gkeys, [[(idx[k1], pt) for k1, pt in terms[k2]]
                                                    for k2 in giants])
        ks = sorted({k1 for tl in plan["terms"].values() for k1, _ in tl if k1})
        baby = {0: ct}
        if ks:
            rots = e.rotate_hoisted(ct, [self.hrot[(k1 * u) % self.n] for k1 in ks])
            baby.update(zip(ks, rots))
        out = None
        for k2, tl in sorted(plan["terms"].items()):
            part = e.dot_plain([baby[k1] for k1, _ in tl], [pt for _, pt in tl])
            part = self._rot(part, g * k2 * u)
            out = part if out is None else e.add(out, part)
        return out

    def chebyshev(self, x: Ciphertext, coeffs: np.ndarray | None = None) -> Ciphertext:
        """sum_k c_k T_k(x) by recursive Chebyshev division (baby steps T_1..T_b, giants
        T_2b, T_4b, ...): for d >= g (g the largest giant <= d),
        p = q T_g + r with T_{g+j} = 2 T_g T_j - T_{g-j}, so q_0 = c_g, q_j = 2 c_{g+j},
        r_{g-j} -= c_{g+j}; leaves (degree < b) are one lincomb of T_1..T_{b-1}.  For deg 31,
        b = 8: 11 ciphertext products (T_2..T_8, T_16, three splits) instead of 30, same depth
        ceil(log2(deg + 1)) + 1, and 10 relinearisations (the top split's product shares one
        with its remainder's)."""
        e = self.e
        cheb = self.cheb if coeffs is None else coeffs
        deg = len(cheb) - 1
        T = {1: x}

        def tk(k):
            if k not in T:
                a = 1 << (k.bit_length() - 1)
                if a == k:
                    a = k // 2
                b = k - a
                # T_{a+b} = 2 T_a T_b - T_{a-b} (T_0 = 1): one fused multiply-add
                if a == b:
                    T[k] = e.multiply_fma(tk(a), tk(b), self.rlk, alpha=2, beta=-1.0)
                else:
                    T[k] = e.multiply_fma(tk(a), tk(b), self.rlk, alpha=2, c=tk(a - b), gamma=-1.0)
            return T[k]

        baby = 1 << max(1, (deg + 1).bit_length() // 2)  # 8 for deg 31, 4 for deg 15

        # ev returns the value as (pairs, lin, c0) = sum a_i b_i + lin + c0 with the products not
        # yet relinearised: a node's own giant product joins its remainder's pending products, so
        # the products summed into one value share ONE relinearisation + rescale (Engine.dot) --
        # deg 31: 2 giant relinearisations instead of 3, same depth.
        def materialize(pairs, lin, c0):
            out = e.dot([a for a, _ in pairs], [b for _, b in pairs], self.rlk) if pairs else None
            if lin is not None:
                out = lin if out is None else e.add(out, lin)
            return out, c0

        def ev(c):
            d = len(c) - 1
            while d > 0 and abs(c[d]) < 1e-14:
                d -= 1
            if d < baby:
                ks = [k for k in range(1, d + 1) if abs(c[k]) > 1e-14]
                out = e.lincomb([tk(k) for k in ks], [complex(c[k]) for k in ks]) if ks else None
                return [], out, complex(c[0])
            g = baby
            while 2 * g <= d:
                g *= 2
            q = np.zeros(d - g + 1)
            r = np.array(c[:g], dtype=float)
            q[0] = c[g]
            for jj in range(1, d - g + 1):
                q[jj] = 2.0 * c[g + jj]
                r[g - jj] -= c[g + jj]
            qc, q0 = materialize(*ev(q))
            rp, rl, r0 = ev(r)
            qt = e.add(qc, q0) if qc is not None else None
            if qt is None:
                prod = e.multiply(tk(g), q0)
                return rp, (prod if rl is None else e.add(prod, rl)), r0
            return [(qt, tk(g))] + rp, rl, r0

        out, c0 = materialize(*ev(list(cheb)))
        T.clear()  # ev / tk form a closure cycle: release the T_k now, not at the next gc pass
        return e.add(out, c0)

    def chebyshev_opt(self, x: Ciphertext, coeffs: np.ndarray) -> Ciphertext:
        """sum_k c_k T_k(x) in depth ceil(log2(deg + 1)) -- one level less than `chebyshev`.

        Canonical scales make every non-integer constant cost a level, so a leaf
        c_0 + ... + c_7 T_7 cannot sit at depth 3.  Here the leaves stop at degree 3 and take
        their constants where a level is free: c_3 T_3 = T_2 (2 c_3 T_1) - c_3 T_1 gives
            c_0 + c_1 T_1 + c_2 T_2 + c_3 T_3 = c_0 + (c_1 - c_3) T_1 + c_2 T_2 + T_2 (2 c_3 T_1)
        (T_2 and the depth-1 multiple of x multiply at depth 2 = ceil(log2 4)); above the leaves
        the same recursive division as `chebyshev` by the giants T_4, T_8, T_16, ..
        (T_2g = 2 T_g^2 - 1): p = q T_g + r with deg q < g lands at depth log2(g) + 1.

        Every part is produced at the level where it is consumed (`ev(c, lv)`): a node's
        products are (a, b) pairs with both operands at lv + 1, summed by ONE relinearisation
        together with its remainder's pairs, its linear terms (x, T_2, T_g with constants, read
        truncated with their scale folded into the constant) and its constant: one
        aesfhe_dot_fma per materialised node.  The depth-1 multiples of x are lincombs that land
        at the level they are used at; the giants are level-downed once per level needed.
        Degree 15: 7 relinearisations (3 of them the giants T_2, T_4, T_8), depth 4; degree 29:
        11 (4 giants), depth 5."""
        e = self.e
        l0 = x.level
        T = {1: x}
        down = {}
        marks = {}
        tiny = 1e-14

        def giant(g, lv=None):
            if g not in T:
                h = giant(g // 2)
                T[g] = e.multiply_fma(h, h, self.rlk, alpha=2, beta=-1.0)
            t = T[g]
            if lv is None or t.level == lv:
                return t
            if (g, lv) not in down:
                down[(g, lv)] = e.level_down(t, lv)
            return down[(g, lv)]

        def lincomb_at(terms, lv):
            """sum k * ct as one lincomb whose output is at level lv (a zero marker ciphertext
            at lv + 1 sets the level when every input sits higher)."""
            cts = [c for c, _ in terms]
            ks = [complex(k) for _, k in terms]
            if min(c.level for c in cts) - 1 > lv:
                if lv + 1 not in marks:
                    marks[lv + 1] = e.zeros(1, lv + 1)
                cts.append(marks[lv + 1])
                ks.append(0j)
            return e.lincomb(cts, ks)

        def lin_add(lin, g, k):
            if abs(k) >= tiny:
                lin[g] = lin.get(g, 0.0) + k

        def materialize(pairs, lin, c0, lv):
            terms = [(giant(g), k) for g, k in sorted(lin.items())]
            if pairs:  # products, linear terms and constant: one aesfhe_dot_fma
                return e.dot_fma([a for a, _ in pairs], [b for _, b in pairs], self.rlk, terms, c0)
            if not terms:
                raise ValueError("chebyshev_opt: constant node")
            y = lincomb_at(terms, lv)
            return e.add(y, c0) if c0 != 0 else y

        def ev(c, lv):
            """(pairs with operands at lv + 1, {giant g: coefficient} for a lincomb at lv, c_0)"""
            d = len(c) - 1
            while d > 0 and abs(c[d]) < tiny:
                d -= 1
            lin = {}
            if d <= 3:
                pairs = []
                if d == 3:
                    lam = lincomb_at([(x, 2.0 * c[3])], lv + 1)
                    pairs.append((giant(2, lv + 1), lam))
                    lin_add(lin, 1, float(c[1] - c[3]))
                elif d >= 1:
                    lin_add(lin, 1, float(c[1]))
                if d >= 2:
                    lin_add(lin, 2, float(c[2]))
                return pairs, lin, float(c[0])
            g = 1 << (d.bit_length() - 1)
            q = np.zeros(d - g + 1)
            r = np.array(c[:g], dtype=float)
            q[0] = c[g]
            for j in range(1, d - g + 1):
                q[j] = 2.0 * c[g + j]
                r[g - j] -= c[g + j]
            pairs, lin, r0 = ev(r, lv)
            if d == g:
                lin_add(lin, g, float(q[0]))  # q is the constant c_g
            else:
                qt = materialize(*ev(q, lv + 1), lv + 1)
                pairs = pairs + [(qt, giant(g, lv + 1))]
            return pairs, lin, r0

        deg = len(coeffs) - 1
        out = materialize(*ev(list(coeffs), l0 - math.ceil(math.log2(deg + 1))), l0 - math.ceil(math.log2(deg + 1)))
        T.clear()
        down.clear()
        marks.clear()
        return out

    def evalmod(self, x: Ciphertext, bits: bool = False) -> Ciphertext:
        e = self.e
        if bits and self.bits_opt:
            c = self.chebyshev_opt(x, self.cheb_bits)
        else:
            c = self.chebyshev(x, self.cheb_bits if bits else self.cheb)
        for _ in range(self.bits_r if bits else self.r):
            c = e.multiply_fma(c, c, self.rlk, alpha=2, beta=-1.0)  # cos 2t = 2 cos^2 t - 1
        return c  # sin(2 pi Bnd x)

    def _raise_to_slots(self, c: Ciphertext, bits: bool = False):
        """Level-0 ciphertext (coefficients t mod q0) -> (x_re, x_im) with slots t / (q0 Bnd) of
        the bit-reversed real / imaginary coefficient halves, at level L - 1 - groups (bit mode
        with bits_opt: L - groups, c_in folded into the CtS diagonals)."""
        e = self.e
        c = e.switch_key(c, self.to_sparse)
        c = e.mod_raise(c, self.L)
        c = e.switch_key(c, self.from_sparse)
        if bits and self.bits_opt:
            plans = self.cts_bits
        else:
            c = e.multiply(c, self.c_in)
            plans = self.cts
        for plan in plans:
            c = self.linear(c, plan)
        cj = e.conjugate(c, self.cjk)
        return e.add(c, cj), e.multiply_i(e.subtract(c, cj), -1)

    def plan_keys(self, plan) -> list:
        """The rotation keys a linear map's plan switches with (babies, then giants)."""
        u, g = plan["u"], plan["g"]
        ks = {k1 for tl in plan["terms"].values() for k1, _ in tl if k1}
        out = [self.hrot[(k1 * u) % self.n] for k1 in sorted(ks)]
        out += [self.rot[(g * k2 * u) % self.n] for k2 in sorted(plan["terms"]) if (g * k2 * u) % self.n]
        return out

    def bootstrap(self, ct: Ciphertext) -> Ciphertext:
        """General complex slots (CtS -> EvalMod -> StC): output at level L - depth."""
        if getattr(self, "_bits_only", False):
            raise RuntimeError("this bootstrapper's SlotToCoeff keys were trimmed for the bit mode "
                               "(trim_bootstrap_keys): general bootstrapping needs them whole")
        e = self.e
        c = ct if ct.level == 0 else e.level_down(ct, 0)
        x_re, x_im = self._raise_to_slots(c)
        nb = x_re.batch
        ys = self.evalmod(e.concat([x_re, x_im]))  # one batched evaluation for both halves
        y = e.add(e.slice(ys, 0, nb), e.multiply_i(e.slice(ys, nb, nb), 1))
        for plan in self.stc:
            y = self.linear(y, plan)
        return y

    def _stc_bits_for(self, in_scale: float):
        """SlotToCoeff plans for inputs holding in_scale * (+-1): the last map's constant divided
        by in_scale (plaintext constants only: no level), prepared on first use."""
        key = float(in_scale)
        if key not in self._stc_bits_scaled:
            last = {d: v / key for d, v in self._stc_bits_maps[-1].items()}
            self._stc_bits_scaled[key] = self.stc_bits[:-1] + [self._prepare(last, self.stc_baby_scale)]
        return self._stc_bits_scaled[key]

    def bootstrap_bits(self, a: Ciphertext, b: Ciphertext | None = None, in_scale: float = 1.0):
        """Refresh one or two ciphertexts whose real slots hold bits +-1 (SlotToCoeff first).
        in_scale: the inputs hold in_scale * (+-1) instead (AESRowRound.clean_bits' 3x - x^3 =
        2 x (3 - x^2) / 2): SlotToCoeff's last constant absorbs the factor.

        StC at the bottom levels puts the bits into the coefficients as +-q0/4 (a in the first
        half, b in the second); after ModRaise t/q0 = I +- 1/4 + eps, so EvalMod's
        sin(2 pi t / q0) = +-cos(2 pi eps) returns the bits in the slots directly -- the
        error of the input bits enters squared, and the signal is O(1) (no q0 / D_0 gain at the
        end).  Inputs need level >= groups; outputs are at ``self.bits_level`` = L - 11 with the
        defaults (L - 13 with bits_opt=False).  Returns (a', b') (b' None when b is None)."""
        e = self.e
        lv = len(self.stc_bits)
        x = a if b is None else e.add(e.level_down(a, min(a.level, b.level)),
                                       e.multiply_i(e.level_down(b, min(a.level, b.level)), 1))
        if x.level < lv:
            raise ValueError(f"bootstrap_bits needs level >= {lv}, got {x.level}")
        if x.level > lv:
            x = e.level_down(x, lv)
        for plan in self._stc_bits_for(in_scale):
            x = self.linear(x, plan)
        x_re, x_im = self._raise_to_slots(x, bits=True)
        if b is None:
            return self.evalmod(x_re, bits=True), None
        nb = x_re.batch
        ys = self.evalmod(e.concat([x_re, x_im]), bits=True)  # one batched evaluation for both halves
        return e.slice(ys, 0, nb), e.slice(ys, nb, nb)


def trim_bootstrap_keys(bss) -> int:
    """For drivers that refresh bits only (bootstrap_bits: the AES flows): trim every rotation key
    that no CoeffToSlot map of any of these bootstrappers uses to the SlotToCoeff levels.  In the
    bit mode SlotToCoeff runs at levels len(stc_bits) .. 1 (bootstrap_bits levels its input down
    to len(stc_bits) first), where a key switch reads one digit of the dnum (Engine.trim_key: the
    kept digit is the full key's word for word, results unchanged).  CoeffToSlot keys switch at
    the top levels and stay whole; keys shared between bootstrappers (share=) count every use.
    General bootstrapping then refuses (its SlotToCoeff runs high).  Returns the bytes freed.
    Config 5 (N = 2^17, 48 limbs, 3 digits): 0.3 GB per key before, 0.1 GB after."""
    if not bss:
        return 0
    e = bss[0].e
    top = {}   # id(key) -> (key, highest level it switches at)
    for bs in bss:
        for plans, lv in ((bs.cts + (bs.cts_bits if bs.cts_bits is not bs.cts else []), bs.L),
                          (bs.stc_bits, len(bs.stc_bits))):
            for plan in plans:
                for k in bs.plan_keys(plan):
                    old = top.get(id(k))
                    top[id(k)] = (k, max(lv, old[1] if old else -1))
    before = after = 0
    for k, lv in top.values():
        b0 = e.key_bytes(k)
        if lv < e.max_level:
            e.trim_key(k, lv)
        before += b0
        after += e.key_bytes(k)
    for bs in bss:
        bs._bits_only = True
    return before - after
