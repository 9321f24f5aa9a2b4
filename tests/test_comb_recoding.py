"""CPU: the index arithmetic of the HBM wide combs, restated on the host.

* coa_smul.h wc_recode / wc_take_digit: a scalar x < 2^(W POS - 1) becomes
  POS signed W-bit digits d_j with sum d_j 2^(W j) == x and |d_j| <= 2^(W-1)
  -- for B's comb (W 24, POS 11: any s < 2^256) and the keys' combs (W 20,
  POS 13; W 16, POS 16: k < l).
* For the keys (k < l), the top radix-2^20 digit is at most 2^13, which is
  what lets k_key_wcomb20 leave the entries (12, m > 2^16) unbuilt.
* coa_committee.hip k_key_wcomb20: entry (j, m) = m 2^(20 j) is the sum of the
  radix-256 comb entries (q, b0), (q+1, b1), (q+2, b2) with signed bytes
  |b_i| <= 128 (the radix-256 comb's range) and q + 2 <= 31 wherever a digit
  can reach it."""
import random

import pytest

L_ORDER = 2**252 + 27742317777372353535851937790883648493


def wc_digits(x, W, POS):
    """wc_recode + POS x wc_take_digit (coa_smul.h)."""
    r = x + sum(1 << (W * j + W - 1) for j in range(POS))
    out = []
    for _ in range(POS):
        out.append((r & ((1 << W) - 1)) - (1 << (W - 1)))
        r >>= W
    return out


def key_wcomb20_bytes(j, m):
    """k_key_wcomb20's decomposition of m * 2^(20 j) into (position, byte)."""
    bit = 20 * j
    q, v = bit >> 3, m << (bit & 7)
    bs, carry = [], 0
    for i in range(3):
        x = (v & 255) + carry
        v >>= 8
        carry = 0
        if i < 2 and x >= 128:
            x -= 256
            carry = 1
        bs.append(x)
    return q, bs


@pytest.mark.parametrize("W,POS", [(24, 11), (20, 13), (16, 16)])
def test_wide_comb_digits(W, POS):
    rng = random.Random(W)
    xs = [0, 1, L_ORDER - 1, 2**253 - 1, 2**256 - 1] + [rng.getrandbits(256) for _ in range(400)]
    # every x the kernels recode: B's comb takes any s < 2^256 (W POS = 264),
    # the 2^16 key comb only k < l (W POS = 256 covers x < 2^255)
    for x in (x for x in xs if x < 1 << (W * POS - 1)):
        d = wc_digits(x, W, POS)
        assert sum(dj << (W * j) for j, dj in enumerate(d)) == x
        assert all(-(1 << (W - 1)) <= dj <= (1 << (W - 1)) for dj in d)


def test_key_top_digit_bound():
    rng = random.Random(5)
    for k in [0, L_ORDER - 1] + [rng.randrange(L_ORDER) for _ in range(2000)]:
        assert abs(wc_digits(k, 20, 13)[12]) <= 1 << 13


def test_key_wcomb20_entries():
    rng = random.Random(9)
    for j in range(13):
        ms = [1, 2, 127, 128, 129, 255, 256, (1 << 13), (1 << 16), (1 << 19) - 1, 1 << 19]
        ms += [rng.randrange(1, (1 << 19) + 1) for _ in range(300)]
        for m in ms:
            q, bs = key_wcomb20_bytes(j, m)
            assert all(-128 <= b <= 128 for b in bs)
            used = [(q + i, b) for i, b in enumerate(bs) if b]
            value = sum(b << (8 * p) for p, b in used)
            if j < 12 or m <= 1 << 13:  # every entry a key's digit can select
                assert all(p <= 31 for p, _ in used)
                assert value == m << (20 * j)
            else:  # never read (test_key_top_digit_bound): position 32 may be needed
                assert value == m << (20 * j) or any(p > 31 for p, _ in used)
