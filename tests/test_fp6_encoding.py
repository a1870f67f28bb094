"""CPU checks of the arithmetic behind k_gemm9 (csrc/q4_0_gemm.hip `e2m3_half`, `f6_pack`):
the block-scaled fp6 MFMA computes the exact q4_0 x q8_0 block sum when

  weights  w = nibble - 8 in [-8, 7] enter as the e2m3 value w/2 with block scale 2^1, and
  x        q in [-128, 127] enters as (q >> 4)/2 with scale 2^5 in K half 0 and (q & 15)/2 with scale 2^1
           in K half 1,

because every such half-integer is an e2m3 value (1 sign, 2 exponent bits with bias 1, 3 mantissa bits)
and 2*(w/2) * (16*(q >> 4) + (q & 15)) = w*q.  Here the device encoder is restated in numpy, decoded
by the e2m3 definition, and the packed 6-bit layout is checked to round-trip.  (The hardware side, the
operand lane maps and the exactness of the instruction on every code, is tools/fp6_check.hip on the GPU
and the bitwise k_gemm9 == k_gemm8 tests in test_gpu_parity.py.)"""
import numpy as np


def e2m3_half(n):
    """the device encoder: e2m3 code of n/2 for integer n in [-15, 15]"""
    a = abs(n)
    c = 4 * a if a < 4 else (8 + 2 * a if a < 8 else 16 + a)
    return (0x20 if n < 0 else 0) | c


def e2m3_value(code):
    """OCP e2m3 definition: sign bit 5, exponent bits 4..3 (bias 1), mantissa bits 2..0; no inf / nan"""
    s = -1.0 if code & 0x20 else 1.0
    e = (code >> 3) & 3
    m = code & 7
    return s * (m / 8.0 if e == 0 else 2.0 ** (e - 1) * (1.0 + m / 8.0))


def test_every_half_integer_in_range_is_exact():
    for n in range(-15, 16):
        assert e2m3_value(e2m3_half(n)) == n / 2.0, n


def test_codes_are_six_bits_and_distinct():
    codes = [e2m3_half(n) for n in range(-15, 16)]
    assert all(0 <= c < 64 for c in codes)
    assert len(set(codes)) == len(codes)                     # n = 0 is +0; no -0 is produced
    assert e2m3_half(0) == 0


def test_split_reproduces_every_q8_value():
    for q in range(-128, 128):
        hi, lo = q >> 4, q & 15
        assert -8 <= hi <= 7 and 0 <= lo <= 15
        vh, vl = e2m3_value(e2m3_half(hi)), e2m3_value(e2m3_half(lo))
        assert vh * 2.0 ** 5 + vl * 2.0 ** 1 == q                # the two K halves with their block scales


def test_block_sum_identity_on_random_blocks():
    rng = np.random.default_rng(5)
    for _ in range(200):
        w = rng.integers(-8, 8, 32)
        q = rng.integers(-128, 128, 32)
        ww = np.array([e2m3_value(e2m3_half(int(v))) for v in w]) * 2.0          # scale 2^1
        xh = np.array([e2m3_value(e2m3_half(int(v) >> 4)) for v in q]) * 2.0 ** 5
        xl = np.array([e2m3_value(e2m3_half(int(v) & 15)) for v in q]) * 2.0
        s = float(np.dot(ww, xh) + np.dot(ww, xl))
        assert s == float(np.dot(w, q))
        assert abs(s) < 2 ** 24                                # every partial sum exact in f32


def f6_pack(codes):
    """the device packer: 32 codes -> 6 dwords, element j at bits 6j .. 6j+5"""
    F = [codes[4 * m] | codes[4 * m + 1] << 6 | codes[4 * m + 2] << 12 | codes[4 * m + 3] << 18 for m in range(8)]
    D = [F[0] | (F[1] << 24), (F[1] >> 8) | (F[2] << 16), (F[2] >> 16) | (F[3] << 8),
         F[4] | (F[5] << 24), (F[5] >> 8) | (F[6] << 16), (F[6] >> 16) | (F[7] << 8)]
    return [d & 0xFFFFFFFF for d in D]


def test_pack_layout_round_trips():
    rng = np.random.default_rng(9)
    for _ in range(100):
        codes = [int(c) for c in rng.integers(0, 64, 32)]
        bits = sum(d << (32 * i) for i, d in enumerate(f6_pack(codes)))
        assert [(bits >> (6 * j)) & 63 for j in range(32)] == codes


def e2m3_half_branchfree(n):
    """the device encoder as compiled (csrc/q4_0_gemm.hip e2m3_half): e = (a >= 4) + (a >= 8),
    c = (a << (2 - e)) + 8e, sign from bit 31 of n"""
    a = abs(n)
    e = int(a >= 4) + int(a >= 8)
    return (((n & 0xFFFFFFFF) >> 26) & 0x20) | ((a << (2 - e)) + 8 * e)


def test_branchfree_encoder_equals_definition():
    for n in range(-15, 16):
        assert e2m3_half_branchfree(n) == e2m3_half(n), n


def g9_tile(i, G, Mt, ny, xcd):
    """k_gemm9's workgroup id -> (row tile, token tile) (csrc/q4_0_gemm.hip, G9Mats.xcd)"""
    j = i
    if xcd:
        C = G >> 3
        if j < 8 * C:
            j = (j & 7) * C + (j >> 3)
        rt = j // ny
        return rt, j - rt * ny
    return j % Mt, j // Mt


def test_g9_tile_order_is_a_permutation_and_xcd_local():
    """Every tile exactly once in both orders; in the XCD-aware order (workgroup i runs on XCD i % 8)
    each XCD gets a contiguous row-tile-major range, so the token tiles of a row tile share one XCD
    except at the at most 7 range boundaries."""
    for Mt, ny in [(32, 8), (86, 8), (96, 8), (172, 8), (3, 1), (13, 1), (7, 4), (35, 3), (1, 1)]:
        G = Mt * ny
        for xcd in (0, 1):
            tiles = [g9_tile(i, G, Mt, ny, xcd) for i in range(G)]
            assert sorted(tiles) == [(r, t) for r in range(Mt) for t in range(ny)], (Mt, ny, xcd)
        xcds = {}
        for i in range(G):
            xcds.setdefault(g9_tile(i, G, Mt, ny, 1)[0], set()).add(i % 8)
        split = sum(len(s) > 1 for s in xcds.values())
        if G >= 8:
            assert split <= 7, (Mt, ny, split)
        if G % 8 == 0 and (G // 8) % ny == 0:
            assert split == 0, (Mt, ny)


def e2m3_tab4(n0):
    """csrc/q4_0_device.h e2m3_tab4: the codes of n0 .. n0 + 3, one per byte"""
    return sum(e2m3_half(n0 + i) << (8 * i) for i in range(4))


def v_perm_b32(s0, s1, sel):
    """V_PERM_B32 for selector bytes 0..7: byte i of the result = byte sel_i of the 64-bit {s0 (high), s1 (low)}"""
    src = (s0 << 32) | s1
    return sum(((src >> (8 * ((sel >> (8 * i)) & 0xFF))) & 0xFF) << (8 * i) for i in range(4))


def e2m3_codes4(idx, u0, u1):
    """csrc/q4_0_device.h e2m3_codes4: four 4-bit indices (one per byte) -> four codes"""
    sel = idx & 0x07070707
    r0 = v_perm_b32(e2m3_tab4(4), e2m3_tab4(0), sel)
    r1 = v_perm_b32(u1, u0, sel)
    m = (((idx >> 3) & 0x01010101) * 0xFF) & 0xFFFFFFFF
    return (r1 & m) | (r0 & ~m & 0xFFFFFFFF)


def f6x4_bytes(c):
    return (c & 0x3F) | ((c >> 2) & 0xFC0) | ((c >> 4) & 0x3F000) | ((c >> 6) & 0xFC0000)


def test_byte_table_encoder_equals_per_element_encoder():
    """x9_store_lane's lookups (packed >> 4 with the n = -8..-1 table for q >> 4, packed with 8..15 for
    q & 15) give the per-element e2m3_half fields for every q8 value in every byte position"""
    rng = np.random.default_rng(11)
    qs = [list(range(-128, 128))[i:i + 4] for i in range(0, 256, 4)] + \
         [[int(v) for v in rng.integers(-128, 128, 4)] for _ in range(2000)]
    for q in qs:
        packed = sum((v & 0xFF) << (8 * i) for i, v in enumerate(q))
        fh = f6x4_bytes(e2m3_codes4(packed >> 4, e2m3_tab4(-8), e2m3_tab4(-4)))
        fl = f6x4_bytes(e2m3_codes4(packed, e2m3_tab4(8), e2m3_tab4(12)))
        hi = [e2m3_half(v >> 4) for v in q]
        lo = [e2m3_half(v & 15) for v in q]
        assert fh == hi[0] | hi[1] << 6 | hi[2] << 12 | hi[3] << 18, q
        assert fl == lo[0] | lo[1] << 6 | lo[2] << 12 | lo[3] << 18, q
