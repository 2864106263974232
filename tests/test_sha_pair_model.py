"""CPU model of the lane-pair SHA-256 compression (celestia-app_amd/csrc/
sha256_dev.h sha_pair_compress): two lanes run one instruction stream, the
e-side lane holding (e, f, g, h), the a-side lane (a, b, c, d); per-lane
rotate amounts, a select for Ch / Maj and a partner swap for T1 and d.  The
model executes the same per-lane operations step by step and must equal
hashlib on random messages (the GPU kernels using it are checked against the
oracle by the -m gpu suite)."""
import hashlib
import struct

import numpy as np

M32 = 0xFFFFFFFF
K = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def pair_compress(lanes, w):
    """lanes[0] = e-side [e f g h] state, lanes[1] = a-side [a b c d]; w: 16
    message words, identical in both lanes (each lane keeps its own copy)."""
    w = [list(w), list(w)]
    r = [(6, 11, 25), (2, 13, 22)]          # Sigma1 / Sigma0 per lane
    q = [(17, 19, 10), (7, 18, 3)]          # sigma1 / sigma0 per lane
    v = [list(lanes[0]), list(lanes[1])]
    for i in range(64):
        if i < 16:
            wi = [w[0][i], w[1][i]]
        else:
            # x = pair_sel(w[t-2], w[t-15]); sg = per-lane sigma; w[t] = u + sg(partner)
            x = [w[0][(i - 2) & 15], w[1][(i - 15) & 15]]
            sg = [rotr(x[L], q[L][0]) ^ rotr(x[L], q[L][1]) ^ (x[L] >> q[L][2]) for L in (0, 1)]
            u = [(sg[L] + w[L][(i - 7) & 15] + w[L][i & 15]) & M32 for L in (0, 1)]
            wi = [(u[0] + sg[1]) & M32, (u[1] + sg[0]) & M32]
            for L in (0, 1):
                w[L][i & 15] = wi[L]
        S = [rotr(v[L][0], r[L][0]) ^ rotr(v[L][0], r[L][1]) ^ rotr(v[L][0], r[L][2]) for L in (0, 1)]
        ch = [(v[L][0] & v[L][1]) ^ (~v[L][0] & v[L][2]) for L in (0, 1)]
        mj = [(v[L][0] & v[L][1]) ^ (v[L][0] & v[L][2]) ^ (v[L][1] & v[L][2]) for L in (0, 1)]
        F = [ch[0] & M32, mj[1]]                                      # pair_sel(ch, maj)
        Y = [(v[0][3] + K[i] + wi[0]) & M32, 0]                       # pair_sel(h + K + W, 0)
        T = [(S[L] + F[L] + Y[L]) & M32 for L in (0, 1)]
        P = [T[0], v[1][3]]                                           # pair_sel(T, v3)
        nv = [(T[0] + P[1]) & M32, (T[1] + P[0]) & M32]               # pair_add(T, P)
        for L in (0, 1):
            v[L] = [nv[L], v[L][0], v[L][1], v[L][2]]
    return [[(lanes[L][j] + v[L][j]) & M32 for j in range(4)] for L in (0, 1)]


def sha256_pair(msg: bytes) -> bytes:
    ml = len(msg) * 8
    msg = msg + b"\x80" + b"\x00" * ((55 - len(msg)) % 64) + struct.pack(">Q", ml)
    lanes = [IV[4:], IV[:4]]
    for off in range(0, len(msg), 64):
        lanes = pair_compress(lanes, struct.unpack(">16I", msg[off:off + 64]))
    return struct.pack(">8I", *(lanes[1] + lanes[0]))   # sha_pair_digest: H0..H3 (a-side), H4..H7


def test_pair_model_equals_sha256():
    rng = np.random.default_rng(7)
    for n in (0, 1, 55, 56, 64, 65, 91, 181, 542):   # empty, padding edges, RFC leaf/inner, NMT node, leaf
        for _ in range(3):
            m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert sha256_pair(m) == hashlib.sha256(m).digest(), n
