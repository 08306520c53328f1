"""VALU estimate per dword column (4 bytes of every shard) of the two GF(2^8) encode forms:
the v_perm table multiply (gf_device.hpp: 5 VALU of bit groups per input dword, then 3 perms
+ 1.5 XOR3 + 0.25 table moves per coefficient) and the compiled bit-plane network
(gf_bitslice.hpp: 6 VALU of transpose per dword of every shard, then one XOR3 per two terms
of each output plane).  Terms come from the parity rows of reedsolomon.go buildMatrix via
the oracle's restatement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.rs_numpy import build_matrix, gf_mul  # noqa: E402


def ones(c):
    # bit p of c * 2^q over all (p, q): the coefficient's 8x8 bit matrix
    return sum(bin(gf_mul(c, 1 << q)).count("1") for q in range(8))


for k, m in ((3, 2), (4, 2), (6, 3), (8, 3), (10, 4), (12, 5)):
    P = build_matrix(k, m)[k:]
    terms = [[sum((gf_mul(int(P[r][c]), 1 << q) >> p) & 1 for c in range(k) for q in range(8)) for p in range(8)]
             for r in range(m)]
    net = (sum((t - 1 + 1) // 2 for row in terms for t in row) + 6 * 8 * (k + m)) / 8
    perm = 5 * k + m * k * 4.75
    print(f"RS({k},{m}): ones/coef {sum(ones(int(c)) for c in P.flat) / (k * m):.1f}  "
          f"VALU per dword column: network {net:.1f}, v_perm tables {perm:.1f} ({net / perm:.2f}x)")
