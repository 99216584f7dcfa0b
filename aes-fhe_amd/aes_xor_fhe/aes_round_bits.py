"""Row-sliced, bit-domain homomorphic AES-128 round (the fast path of the bench).

Same primitive kinds as the reference's services (LUT polynomials as in xor_service.py:245-286
/ sbox_service.py:116-138, slot rotations as in shiftrows_service.py:33-51), arranged so that
the expensive operations disappear.  The state is carried as +-1 bits B = (-1)^bit:

* layout -- one ciphertext per state row r and bit j: slot = c * n_blk + block with
  n_blk = slot_count / 4 (8192 blocks at N = 2^16).  ShiftRows (out(r,c) = in(r, c+r)) is a
  single whole-ciphertext rotation of row r by -r*n_blk slots, no masks (24 per 8192 blocks),
  applied to the SubBytes output (it commutes with SubBytes; 4 levels lower = fewer limbs).
* SubBytes -- every Boolean function of a byte is a multilinear polynomial in its +-1 bits
  whose coefficients are its Walsh spectrum.  With M^hi_S / M^lo_T the 15 non-empty monomials
  of the high / low nibble bits (11 products each, depth 2), the 8 output bits are
  out_t = sum_{S,T} W_t[S,T] M^hi_S M^lo_T: one fused Engine.poly2_int call per row (64 W is
  an integer in [-8, 8]: exact integer inner sums, one relinearisation per output bit), depth 2.
* MixColumns + AddRoundKey -- XOR is multiplication.  With a_r the SubBytes bytes of row r and
  U_r = a_r ^ a_{r+1}: out_r = xtime(a_r ^ a_{r+1}) ^ a_{r+1} ^ a_{r+2} ^ a_{r+3}
  = xtime(U_r) ^ U_{r+1} ^ a_{r+3}; xtime(u)_j = u_{j-1} (j = 0: u_7), times u_7 for j in
  {1, 3, 4}.  The round-key bit (B = 1, broadcast) joins a_{r+3} at depth 0:
  out_rj ^ k_rj = xtime(U_r)_j * (U_{r+1,j} * (a_{r+3,j} * K_rj)): 32 + 12 + 96 = 140
  products, depth 3 (plain MixColumns alone: 108 products, depth 3).
Round depth 4 + 3 = 7 (four rounds per 30-level budget); 24 + 88 + 4 + 140 = 256 key switches
per 8192 blocks against ~960 for the byte-major nibble-domain round (aes_round.py).

Full AES-128 (`encrypt_aes128`, BASELINE configs 4-5): AddRoundKey(k0), rounds 1-9, and the
final round without MixColumns (depth 4 + 1), with bit-mode bootstrapping
(bootstrap.Bootstrapper.bootstrap_bits: two bit ciphertexts per refresh, batched) whenever the
next round would leave fewer levels than SlotToCoeff needs.  At L = 30: ARK0 -> 29, rounds 1-3
-> 8, {refresh -> 19, two rounds -> 5} x 2, refresh -> 19, rounds 8-9 and the final round -> 0:
three refreshes (the bootstrap's output level L - 11).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from . import aes_tables as T
from .fhe import Ciphertext, Engine

XT_OF = {0: (7, False), 1: (0, True), 2: (1, False), 3: (2, True), 4: (3, True), 5: (4, False),
         6: (5, False), 7: (6, False)}  # xtime bit j = u[src] (* u[7] if flagged)


def walsh_sbox() -> np.ndarray:
    """W[t, S, T]: +-1 S-box output bit t as sum_{S,T} W M^hi_S M^lo_T (S, T = 4-bit masks of
    the high / low nibble bits; mask 0 = the constant monomial)."""
    x = np.arange(256)
    f = np.stack([1.0 - 2.0 * ((T.SBOX[x].astype(np.int64) >> t) & 1) for t in range(8)])
    mono = np.array([[np.prod([1 - 2 * ((v >> k) & 1) for k in range(4) if (m >> k) & 1])
                      for v in range(16)] for m in range(16)], dtype=np.float64)  # [mask, nibble]
    hi, lo = x >> 4, x & 15
    return np.einsum("tx,sx,ux->tsu", f, mono[:, hi], mono[:, lo]) / 256.0


class AESRowRound:
    """State: 4 rows x 8 +-1 bit ciphertexts (row r, bit j), each batched over NB sets of
    n_blk blocks."""

    GRANULE = 1  # batch elements a shard across ranks must keep together (parallel.shard_range)

    def __init__(self, engine: Engine, sk, pk, rlk, cjk=None, rotation_keys=None):
        self.e = engine
        self.sk, self.pk, self.rlk, self.cjk = sk, pk, rlk, cjk
        self.sc = engine.slot_count
        self.n_blk = self.sc // 4
        self.W = walsh_sbox()
        self.W64 = np.rint(self.W * 64).astype(np.int32)  # 64 W is an integer in [-8, 8]
        assert np.array_equal(self.W64 / 64.0, self.W)
        if rotation_keys is None:
            rotation_keys = {r: engine.create_fixed_rotation_key(sk, -r * self.n_blk) for r in (1, 2, 3)}
        self.rot_keys = rotation_keys

    # ---- layout -----------------------------------------------------------------------------
    def pack(self, blocks: np.ndarray) -> List[np.ndarray]:
        """(NB, n_blk, 16) bytes -> 4 row arrays (NB, slot_count): slot c*n_blk + blk holds byte
        r + 4c (FIPS order) of block blk."""
        b = np.asarray(blocks, dtype=np.uint8)
        return [np.ascontiguousarray(b[:, :, [r + 4 * c for c in range(4)]].transpose(0, 2, 1)).reshape(b.shape[0], self.sc)
                for r in range(4)]

    def unpack(self, rows: Sequence[np.ndarray], nb: int | None = None) -> np.ndarray:
        n = rows[0].shape[0]  # one set per batch element: nothing padded
        out = np.empty((n, self.n_blk, 16), dtype=np.uint8)
        for r in range(4):
            v = np.asarray(rows[r], dtype=np.uint8).reshape(n, 4, self.n_blk)
            for c in range(4):
                out[:, :, r + 4 * c] = v[:, c, :]
        return out

    # ---- device-resident client path (Engine.encrypt_device / decrypt_device) -----------------
    def encrypt_blocks_device(self, blocks):
        """encrypt_blocks for a (NB, n_blk, 16) uint8 torch tensor on the engine's client device:
        packing, +-1 bit slicing, encoding and encryption all on the device."""
        import torch
        b = blocks.to(self.e.client_device)
        nb = b.shape[0]
        st = []
        for r in range(4):
            row = b[:, :, [r + 4 * c for c in range(4)]].permute(0, 2, 1).reshape(nb, self.sc).to(torch.int64)
            st.append([self.e.encrypt_device(1.0 - 2.0 * ((row >> j) & 1).to(torch.float64), self.pk)
                       for j in range(8)])
        return st

    def decrypt_blocks_device(self, bits, nb: int | None = None):
        """decrypt_blocks into a (NB, n_blk, 16) uint8 torch tensor on the client device."""
        import torch
        rows = []
        for r in range(4):
            acc = None
            for j in range(8):
                v = self.e.decrypt_device(bits[r][j], self.sk).real
                t = (v < 0).to(torch.uint8) << j
                acc = t if acc is None else acc | t
            rows.append(acc)
        nb = rows[0].shape[0]
        out = torch.empty((nb, self.n_blk, 16), dtype=torch.uint8, device=rows[0].device)
        for r in range(4):
            v = rows[r].reshape(nb, 4, self.n_blk)
            for c in range(4):
                out[:, :, r + 4 * c] = v[:, c, :]
        return out

    def encrypt_bytes_rows(self, rows: Sequence[np.ndarray], level: int | None = None):
        return [[self.e.encrypt(1.0 - 2.0 * ((row.astype(np.int64) >> j) & 1), self.pk, level=level)
                 for j in range(8)] for row in rows]

    def encrypt_blocks(self, blocks: np.ndarray, level: int | None = None) -> List[List[Ciphertext]]:
        return self.encrypt_bytes_rows(self.pack(blocks), level=level)

    def decrypt_blocks(self, bits: Sequence[Sequence[Ciphertext]], nb: int | None = None) -> np.ndarray:
        """The state's blocks (NB, n_blk, 16); nb: the number of sets encrypted (a layout that
        pads the batch -- AESSlicedRound -- returns the padding sets too unless told)."""
        rows = []
        for r in range(4):
            acc = 0
            for j in range(8):
                v = np.real(np.atleast_2d(self.e.decrypt(bits[r][j], self.sk)))
                acc = acc | ((v < 0).astype(np.uint8) << j)
            rows.append(acc)
        return self.unpack(rows, nb)

    decrypt_bits = decrypt_blocks

    def encrypt_round_key(self, rk: np.ndarray, level: int | None = None) -> List[List[Ciphertext]]:
        """Key bits as +-1 per row (B = 1, broadcast over the batch)."""
        rk = np.asarray(rk, dtype=np.int64)
        rows = [np.repeat(rk[[r + 4 * c for c in range(4)]], self.n_blk)[None] for r in range(4)]
        return self.encrypt_bytes_rows(rows, level=level)

    # ---- building blocks ---------------------------------------------------------------------
    def mul(self, a: Ciphertext, b: Ciphertext) -> Ciphertext:
        return self.e.multiply(a, b, self.rlk)

    def key_mul(self, a: Ciphertext, k: Ciphertext) -> Ciphertext:
        """a XOR (round-key bit k): the key ciphertext is broadcast over the batch (B = 1)."""
        return self.mul(a, k)

    def monomials(self, b4: Sequence[Ciphertext]) -> Dict[int, Ciphertext]:
        """All 15 non-empty products of 4 +-1 bit ciphertexts, keyed by bit mask (depth <= 2:
        pairs from singles, triples = pair * single, the quadruple = pair * pair)."""
        m = {1 << k: b4[k] for k in range(4)}
        for a in range(4):
            for b in range(a + 1, 4):
                m[(1 << a) | (1 << b)] = self.mul(b4[a], b4[b])
        # the triples multiply a pair (one level down) by a single bit: the engine would align
        # b4[3] to the pairs' level three times over, so it (and b4[2]) is level-downed once here
        # -- the same operation the multiply would run, bit for bit
        lv = min(m[0b0011].level, m[0b0101].level, m[0b0110].level)
        b2, b3 = (c if c.level <= lv else self.e.level_down(c, lv) for c in (b4[2], b4[3]))
        m[0b0111] = self.mul(m[0b0011], b2)
        m[0b1011] = self.mul(m[0b0011], b3)
        m[0b1101] = self.mul(m[0b0101], b3)
        m[0b1110] = self.mul(m[0b0110], b3)
        m[0b1111] = self.mul(m[0b0011], m[0b1100])
        return m

    # ---- round steps ---------------------------------------------------------------------------
    def shift_rows(self, bits):
        return [bits[0]] + [[self.e.rotate(c, self.rot_keys[r]) for c in bits[r]] for r in (1, 2, 3)]

    def sub_bytes(self, bits) -> List[List[Ciphertext]]:
        out = []
        for row in bits:
            mh = self.monomials(row[4:8])
            ml = self.monomials(row[0:4])
            out.append(self.e.poly2_int([mh[i] for i in range(1, 16)], [ml[j] for j in range(1, 16)],
                                        self.W64, 64, self.rlk))
        return out

    def _xtime_terms(self, U, r, j):
        """xtime(u_r) bit j: U[r][j-1] (j = 0: U[r][7]), times U[r][7] for j in {1, 3, 4}."""
        src, carry = XT_OF[j]
        return self.mul(U[r][src], U[r][7]) if carry else U[r][src]

    def mix_columns(self, A: List[List[Ciphertext]]) -> List[List[Ciphertext]]:
        """out_r = xtime(a_r ^ a_{r+1}) ^ a_{r+1} ^ a_{r+2} ^ a_{r+3}
               = xtime(U_r) ^ U_{r+1} ^ a_{r+3},   U_r = a_r ^ a_{r+1}:  108 products, depth 3."""
        U = [[self.mul(A[r][j], A[(r + 1) % 4][j]) for j in range(8)] for r in range(4)]
        return [[self.mul(self._xtime_terms(U, r, j), self.mul(U[(r + 1) % 4][j], A[(r + 3) % 4][j]))
                 for j in range(8)] for r in range(4)]

    def mix_columns_add_round_key(self, A, key) -> List[List[Ciphertext]]:
        """MixColumns then AddRoundKey in one product tree: the key bit joins a_{r+3} first,
        out_rj ^ k_rj = xtime(U_r)_j * (U_{r+1,j} * (a_{r+3,j} * K_rj)): 140 products, depth 3."""
        U = [[self.mul(A[r][j], A[(r + 1) % 4][j]) for j in range(8)] for r in range(4)]
        return [[self.mul(self._xtime_terms(U, r, j),
                          self.mul(U[(r + 1) % 4][j], self.key_mul(A[(r + 3) % 4][j], key[r][j])))
                 for j in range(8)] for r in range(4)]

    def add_round_key(self, S: List[List[Ciphertext]], key) -> List[List[Ciphertext]]:
        return [[self.key_mul(S[r][j], key[r][j]) for j in range(8)] for r in range(4)]

    ROUND_DEPTH, FINAL_DEPTH = 7, 5

    def final_round(self, bits, key):
        """SubBytes -> ShiftRows -> AddRoundKey (AES round 10: no MixColumns), depth 5."""
        return self.add_round_key(self.shift_rows(self.sub_bytes(bits)), key)

    def refresh(self, bits, bs, pairs_per_call: int = 8, in_scale: float = 1.0):
        """Bootstrap all 32 bit ciphertexts, two per refresh (bit j with bit j + 4 of a row),
        `pairs_per_call` pairs concatenated along the batch per Bootstrapper call.  in_scale: the
        bits hold in_scale * (+-1) (clean_bits' output: 2)."""
        e = self.e
        pairs = [(r, j) for r in range(4) for j in range(4)]
        out = [[None] * 8 for _ in range(4)]
        for i in range(0, len(pairs), pairs_per_call):
            grp = pairs[i:i + pairs_per_call]
            nb = bits[0][0].batch
            a = e.concat([bits[r][j] for r, j in grp])
            b = e.concat([bits[r][j + 4] for r, j in grp])
            ya, yb = bs.bootstrap_bits(a, b, in_scale=in_scale)
            for k, (r, j) in enumerate(grp):
                out[r][j] = e.slice(ya, k * nb, nb)
                out[r][j + 4] = e.slice(yb, k * nb, nb)
        return out

    # A round multiplies the slot error of its input by ~10-15 (the S-box's Walsh polynomial sums
    # ~10 products, MixColumns chains three), and bit-mode bootstrapping returns its input error
    # squared: so the error at a refresh must stay ~1e-2.  Measured at N = 2^16 (scale 40,
    # tools/aes10_diag.py, max | |v| - 1 | over all slots): three rounds from a fresh encryption
    # reach 1.8e-3, but a refresh leaves ~1.5e-4, after which two rounds reach 5-7e-3 and a third
    # ~0.1 -- too much for the next refresh (a fourth from a fresh encryption, which L = 35 allows
    # by levels, reached 0.12 at N = 2^17 and the run diverged).  The final round may still follow
    # as a third one: its output is only decrypted (decision margin 1) -- with the last refresh's
    # input cleaned (CLEAN_LEVELS below; without it the margin was not enough, measured 0.7-0.8).
    MAX_ROUNDS_FRESH = 3
    MAX_ROUNDS_AFTER_REFRESH = 2
    # The last refresh is followed by two middle rounds and the final one, and its output error is
    # its input error squared (~pi^2 e^2 / 8): after two middle rounds from the previous refresh
    # the input is ~2.5e-2, the output ~8e-4, and the three rounds after it took the decoded
    # slots to max | |v| - 1 | = 0.7-0.8 at N = 2^16 (round 4: tools/aes10_trace.py) with rare
    # slots past the decision margin 1 -- a wrong block in ~1 of 7 runs of 131 072 blocks.  So
    # the bits are cleaned first, x -> (3x - x^3) / 2 (error e -> ~1.5 e^2, two levels: x^2, then
    # one fused product 3x - x^3 whose factor 2 the refresh's SlotToCoeff absorbs), where the
    # level budget allows it: pick_bootstrapper prefers a previous refresh that leaves the two
    # levels (the 3-map CoeffToSlot one before rounds 6-7 at L = 30).
    CLEAN_LEVELS = 2

    def needs_refresh(self, level: int, final: bool, since: int, refreshed: bool, stc: int) -> bool:
        """Refresh before the next round?  When its depth does not fit, when a middle round would
        leave fewer than `stc` (SlotToCoeff) levels, or after MAX_ROUNDS_* middle rounds."""
        need = self.FINAL_DEPTH if final else self.ROUND_DEPTH
        limit = self.MAX_ROUNDS_AFTER_REFRESH if refreshed else self.MAX_ROUNDS_FRESH
        return level < need or (not final and (level - need < stc or since >= limit))

    def can_clean(self, level: int, since: int, refreshed: bool, stc: int) -> bool:
        """Clean before this refresh?  After MAX_ROUNDS_AFTER_REFRESH middle rounds from a refresh,
        when CLEAN_LEVELS fit above SlotToCoeff's levels (the caller applies it to the last
        refresh only)."""
        return refreshed and since >= self.MAX_ROUNDS_AFTER_REFRESH and level - self.CLEAN_LEVELS >= stc

    def refreshes_after(self, rnd: int, level: int, top: int, stc: int, with_clean: bool = False):
        """Refreshes that rounds rnd..10 need when they start right after a refresh at `level`,
        later refreshes returning `top` (inf if a round would run out of levels).  with_clean:
        (that count, 1 if the last of those refreshes cannot be preceded by clean_bits else 0)."""
        n, since, lvl = 0, 0, level
        last_clean = True
        for r in range(rnd, 11):
            final = r == 10
            if self.needs_refresh(lvl, final, since, True, stc):
                if since == 0:
                    return (float("inf"), 1) if with_clean else float("inf")
                last_clean = self.can_clean(lvl, since, True, stc)
                n, since, lvl = n + 1, 0, top
            lvl -= self.FINAL_DEPTH if final else self.ROUND_DEPTH
            since += 1
            if lvl < 0:
                return (float("inf"), 1) if with_clean else float("inf")
        return (n, 0 if last_clean else 1) if with_clean else n

    def pick_bootstrapper(self, bss, rnd: int):
        """The first of `bss` (cheapest first) whose output level keeps the fewest refreshes for
        rounds rnd..10: a refresh followed by two middle rounds and another refresh needs only
        2 * 7 + StC levels, the one before the last three rounds 7 + 7 + 5."""
        if len(bss) == 1:
            return bss[0]
        stc = len(bss[0].stc_bits)
        top = max(b.bits_level for b in bss)
        # fewest refreshes first, then one that leaves room to clean before the last refresh
        counts = [self.refreshes_after(rnd, b.bits_level, top, stc, with_clean=True) for b in bss]
        return bss[counts.index(min(counts))]

    def refresh_step(self, S, rnd: int, level: int, since: int, refreshed: bool, bss, pairs_per_call: int,
                     probe=None):
        """The refresh before round rnd (state S at `level`, `since` rounds after the previous
        refresh): pick the bootstrapper, clean the bits first when this is the last refresh and
        can_clean allows it, bootstrap.  Returns (state, bootstrapper, cleaned).  probe: optional
        callable(rnd, state, in_scale) shown the state the bootstrap takes (after the cleaning)."""
        stc = len(bss[0].stc_bits)
        b = self.pick_bootstrapper(bss, rnd)
        top = max(x.bits_level for x in bss)
        clean = self.can_clean(level, since, refreshed, stc) and self.refreshes_after(rnd, b.bits_level, top, stc) == 0
        if clean:
            S = self.clean_bits(S)
        if probe is not None:
            probe(rnd, S, 2.0 if clean else 1.0)
        return self.refresh(S, b, pairs_per_call, in_scale=2.0 if clean else 1.0), b, clean

    def bit_margin(self, bits, scale: float = 1.0) -> float:
        """max over every slot of every bit ciphertext of | |v| / scale - 1 |: how far the +-1 bit
        values have drifted (a bit decodes wrongly past 1).  Decrypted on the device when the
        engine is the HIP one (the reduction too), else on the host."""
        worst = 0.0
        for row in bits:
            for c in row:
                if self.e.on_device:
                    v = self.e.decrypt_device(c, self.sk).real
                    d = float((v.abs() / scale - 1.0).abs().max())
                else:
                    v = np.real(np.atleast_2d(self.e.decrypt(c, self.sk)))
                    d = float(np.abs(np.abs(v) / scale - 1.0).max())
                worst = max(worst, d)
        return worst

    def clean_bits(self, bits):
        """3x - x^3 for every bit ciphertext (= 2 * (3x - x^3) / 2, the cleaning map with error
        e -> ~1.5 e^2 near +-1, scaled by 2): x^2, then one fused product -x * x^2 + 3x
        (Engine.multiply_fma), two levels.  The caller's refresh takes in_scale=2."""
        e = self.e
        out = []
        for row in bits:
            sq = [e.multiply(x, x, self.rlk) for x in row]
            out.append([e.multiply_fma(e.level_down(x, y.level) if x.level > y.level else x, y, self.rlk,
                                       alpha=-1, c=x, gamma=3.0) for x, y in zip(row, sq)])
        return out

    KEY_OFFSET = 4  # a round's key product takes the SubBytes output: input level - 4

    def schedule(self, L: int, bss):
        """[(round, input level, bootstrapper refreshing before it or None)] that encrypt_aes128
        runs from a fresh encryption at level L (ARK0 -> L - 1); bss as there (objects with
        bits_level / stc_bits suffice)."""
        bss = list(bss) if isinstance(bss, (list, tuple)) else [bss]
        stc = len(bss[0].stc_bits)
        out, lvl, since, nref = [], L - 1, 0, 0
        for rnd in range(1, 11):
            final = rnd == 10
            b = None
            if self.needs_refresh(lvl, final, since, nref > 0, stc):
                b = self.pick_bootstrapper(bss, rnd)
                lvl, since, nref = b.bits_level, 0, nref + 1
            out.append((rnd, lvl, b))
            lvl -= self.FINAL_DEPTH if final else self.ROUND_DEPTH
            since += 1
        return out

    def fresh_level(self, L: int, bss) -> int:
        """The lowest level a fresh state can be encrypted at (chain top L) whose schedule needs
        no more refreshes than one from L: the first segment's spare levels (at L = 30 it reaches
        its refresh at level 8 where StC needs 3) then go unspent, and its three rounds run on
        fewer limbs -- 25 at L = 30 and at L = 35."""
        def refreshes(s):
            return sum(b is not None for _, _, b in self.schedule(s, bss))
        n, s = refreshes(L), L
        while s > 1 and refreshes(s - 1) == n:
            s -= 1
        return s

    def key_levels(self, L: int, bss) -> List[int]:
        """The level each of the 11 round keys is consumed at (key 0: ARK0 at L; key i: round i's
        SubBytes output level): keys encrypted there need no level-down and hold only the limbs
        they use."""
        return [L] + [lvl - self.KEY_OFFSET for _, lvl, _ in self.schedule(L, bss)]

    def encrypt_aes128(self, bits, keys, bs, timings: dict | None = None, pairs_per_call: int = 8,
                       progress=None, consume: bool = False, probe=None):
        """AES-128 encryption of the bit state under the 11 encrypted round keys `keys`
        (FIPS-197 section 5.1), bootstrapping with `bs` (a bootstrap.Bootstrapper, or a list of them
        cheapest first: each refresh takes the first whose output level costs no extra refresh,
        pick_bootstrapper) as the level budget and the error budget (needs_refresh) require.
        Returns the state and the number of refreshes.  progress: optional callable(str) told
        after each step.  consume: empty the rows of `bits` after AddRoundKey(k_0), so that the
        input state (the largest one, at the top level) is freed if the caller holds it only
        through that list.  probe: optional callable(rnd, state, in_scale) shown every refresh's
        input (refresh_step)."""
        import time
        bss = list(bs) if isinstance(bs, (list, tuple)) else [bs]
        stc = len(bss[0].stc_bits)
        assert all(len(b.stc_bits) == stc for b in bss)
        S = self.add_round_key(bits, keys[0])
        if consume:
            self.e.materialize(S)
            for row in bits:
                row.clear()
        refreshes = 0
        since = 0
        for rnd in range(1, 11):
            final = rnd == 10
            lvl = min(c.level for row in S for c in row)
            if self.needs_refresh(lvl, final, since, refreshes > 0, stc):
                t0 = time.perf_counter()
                S, b, clean = self.refresh_step(S, rnd, lvl, since, refreshes > 0, bss, pairs_per_call, probe)
                since = 0
                refreshes += 1
                if progress:
                    progress(f"refresh {refreshes} before round {rnd} (CtS in {b.cts_groups} maps, output level "
                             f"{b.bits_level}{', bits cleaned first' if clean else ''})")
                if timings is not None:
                    self.e.materialize(S)
                    self.e.synchronize()
                    timings["bootstrap"] = timings.get("bootstrap", 0.0) + time.perf_counter() - t0
            t0 = time.perf_counter()
            lvl = min(c.level for row in S for c in row)
            S = self.final_round(S, keys[rnd]) if final else self.round(S, keys[rnd])
            since += 1
            if progress:
                progress(f"round {rnd} from level {lvl}")
            if timings is not None:
                self.e.materialize(S)  # deferred products belong to this round's time
                self.e.synchronize()
                dt = time.perf_counter() - t0
                timings["rounds"] = timings.get("rounds", 0.0) + dt
                timings.setdefault("per_round", []).append((rnd, lvl, round(1e3 * dt, 1)))
        return S, refreshes

    def round(self, bits, key, timings: dict | None = None):
        """SubBytes -> ShiftRows -> MixColumns -> AddRoundKey on the row-sliced +-1 bit state."""
        import time

        def mark(name, t0, obj=None):
            if timings is None:
                return t0
            self.e.materialize(obj)  # deferred products belong to this stage
            self.e.synchronize()
            t1 = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + (t1 - t0)
            return t1
        t = mark("start", 0.0) if timings is not None else 0.0
        A = self.sub_bytes(bits)  # SubBytes first: ShiftRows commutes with it and is cheaper
        t = mark("sub_bytes", t, A)  # on the SubBytes output (level l-4: fewer limbs per rotation)
        A = self.shift_rows(A)
        t = mark("shift_rows", t, A)
        out = self.mix_columns_add_round_key(A, key)
        mark("mix_columns_add_round_key", t, out)
        return out


class AESSlicedRound(AESRowRound):
    """Fully sliced bit state: the columns move from the slots into the batch.

    One ciphertext per state row r and bit j, as in AESRowRound, but batch element 4 s + c holds
    column c of slab s, one AES block per slot (slot_count = 4 n_blk blocks per slab; the
    external unit stays a set of n_blk blocks, four sets per slab, the last slab zero-padded).
    Every product, the S-box polynomial, MixColumns and the bootstrap are elementwise over the
    batch exactly as before; what changes:

    * ShiftRows, out(r, c) = in(r, c + r), becomes a permutation of row r's batch elements,
      folded into the S-box's output order (aesfhe_poly2_int_rot, sub_bytes_shift_rows): no
      automorphism, no key switch and no copy, where AESRowRound rotates row r by -r n_blk slots
      (24 key switches per 8192 blocks, ~9 % of the round's).
    * The round key differs per column: its ciphertexts carry batch 4 (element c = key byte
      r + 4c); the key product cycles through them (aesfhe_mul: element 4 s + c takes key
      element c), after a level-down of the 4 elements to the state's level (key_mul).
    * The slabs, not the batch elements, are what may be split across ranks (a slab's four
      columns must stay together): a shard of the batch is a multiple of 4 elements
      (GRANULE, parallel.scatter_ciphertext(..., granule=4)).
    """

    GRANULE = 4

    def __init__(self, engine: Engine, sk, pk, rlk, cjk=None, rotation_keys=None):
        super().__init__(engine, sk, pk, rlk, cjk, rotation_keys={})

    # ---- layout -----------------------------------------------------------------------------
    def slabs(self, nb: int) -> int:
        return -(-int(nb) // 4)

    def pack(self, blocks: np.ndarray) -> List[np.ndarray]:
        """(NB, n_blk, 16) bytes -> 4 row arrays (4 S, slot_count), S = ceil(NB / 4) slabs:
        element 4 s + c, slot k holds byte r + 4c (FIPS order) of block k of slab s (the
        blocks of sets 4 s .. 4 s + 3 in order)."""
        b = np.asarray(blocks, dtype=np.uint8)
        nb, S = b.shape[0], self.slabs(b.shape[0])
        flat = np.zeros((S * self.sc, 16), dtype=np.uint8)
        flat[:nb * self.n_blk] = b.reshape(-1, 16)
        sl = flat.reshape(S, self.sc, 16)
        return [np.ascontiguousarray(sl[:, :, [r + 4 * c for c in range(4)]].transpose(0, 2, 1)).reshape(4 * S, self.sc)
                for r in range(4)]

    def unpack(self, rows: Sequence[np.ndarray], nb: int | None = None) -> np.ndarray:
        S = rows[0].shape[0] // 4
        out = np.empty((S, self.sc, 16), dtype=np.uint8)
        for r in range(4):
            v = np.asarray(rows[r], dtype=np.uint8).reshape(S, 4, self.sc)
            for c in range(4):
                out[:, :, r + 4 * c] = v[:, c, :]
        nb = 4 * S if nb is None else int(nb)
        return out.reshape(-1, 16)[:nb * self.n_blk].reshape(nb, self.n_blk, 16)

    def encrypt_blocks_device(self, blocks):
        import torch
        b = blocks.to(self.e.client_device)
        nb, S = b.shape[0], self.slabs(b.shape[0])
        flat = torch.zeros((S * self.sc, 16), dtype=torch.uint8, device=b.device)
        flat[:nb * self.n_blk] = b.reshape(-1, 16)
        sl = flat.reshape(S, self.sc, 16)
        st = []
        for r in range(4):
            row = sl[:, :, [r + 4 * c for c in range(4)]].permute(0, 2, 1).reshape(4 * S, self.sc).to(torch.int64)
            st.append([self.e.encrypt_device(1.0 - 2.0 * ((row >> j) & 1).to(torch.float64), self.pk)
                       for j in range(8)])
        return st

    def decrypt_blocks_device(self, bits, nb: int | None = None):
        import torch
        S = bits[0][0].batch // 4
        out = None
        for r in range(4):
            acc = None
            for j in range(8):
                v = self.e.decrypt_device(bits[r][j], self.sk).real
                t = (v < 0).to(torch.uint8) << j
                acc = t if acc is None else acc | t
            if out is None:
                out = torch.empty((S, self.sc, 16), dtype=torch.uint8, device=acc.device)
            v = acc.reshape(S, 4, self.sc)
            for c in range(4):
                out[:, :, r + 4 * c] = v[:, c, :]
        nb = 4 * S if nb is None else int(nb)
        return out.reshape(-1, 16)[:nb * self.n_blk].reshape(nb, self.n_blk, 16)

    def encrypt_round_key(self, rk: np.ndarray, level: int | None = None) -> List[List[Ciphertext]]:
        """Key bits as +-1 per (row, column): batch 4, element c = key byte r + 4c."""
        rk = np.asarray(rk, dtype=np.int64)
        rows = [np.repeat(rk[[r + 4 * c for c in range(4)]], self.sc).reshape(4, self.sc) for r in range(4)]
        return self.encrypt_bytes_rows(rows, level=level)

    # ---- round steps --------------------------------------------------------------------------
    def key_mul(self, a: Ciphertext, k: Ciphertext) -> Ciphertext:
        """a XOR k: the batch-4 key (element c) against a's elements 4 s + c -- aesfhe_mul's cyclic
        broadcast (element i takes key element i mod 4), so the key is never repeated in memory.
        Aligned to a's level first (the level-down the product would run, on 4 elements)."""
        if k.level > a.level:
            k = self.e.level_down(k, a.level)
        return self.mul(a, k)

    def sub_bytes_shift_rows(self, bits) -> List[List[Ciphertext]]:
        """SubBytes with ShiftRows folded into the S-box polynomial's output order: row r's
        outputs are written rotated by r within each slab (aesfhe_poly2_int_rot) -- no gather, no
        key switch: ShiftRows costs nothing."""
        out = []
        for r, row in enumerate(bits):
            mh = self.monomials(row[4:8])
            ml = self.monomials(row[0:4])
            out.append(self.e.poly2_int([mh[i] for i in range(1, 16)], [ml[j] for j in range(1, 16)],
                                        self.W64, 64, self.rlk, slab_rot=r))
        return out

    def round(self, bits, key, timings: dict | None = None):
        """SubBytes + ShiftRows (one step, sub_bytes_shift_rows) -> MixColumns -> AddRoundKey."""
        import time
        t0 = time.perf_counter()
        A = self.sub_bytes_shift_rows(bits)
        if timings is not None:
            self.e.materialize(A)
            self.e.synchronize()
            t1 = time.perf_counter()
            timings["sub_bytes_shift_rows"] = timings.get("sub_bytes_shift_rows", 0.0) + t1 - t0
        out = self.mix_columns_add_round_key(A, key)
        if timings is not None:
            self.e.materialize(out)
            self.e.synchronize()
            timings["mix_columns_add_round_key"] = timings.get("mix_columns_add_round_key", 0.0) + time.perf_counter() - t1
        return out

    def final_round(self, bits, key):
        """SubBytes + ShiftRows -> AddRoundKey (AES round 10)."""
        return self.add_round_key(self.sub_bytes_shift_rows(bits), key)

    def shift_rows(self, bits):
        """out(r, c) = in(r, c + r): element 4 s + c of row r takes element 4 s + (c + r) mod 4
        (a gather; the round folds it into SubBytes instead, sub_bytes_shift_rows)."""
        S = bits[0][0].batch // 4
        out = [bits[0]]
        for r in (1, 2, 3):
            idx = [4 * s + (c + r) % 4 for s in range(S) for c in range(4)]
            out.append([self.e.gather(c, idx) for c in bits[r]])
        return out
