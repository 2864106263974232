/*
 * cda_oracle.c -- CPU restatement of the celestia-app DA hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so.  The product (celestia-app_amd/, libcda.so) never links it.
 *
 * Restated behaviour (reference paths relative to /root/reference):
 *   - ExtendShares / erasureExtendSquare: pkg/da/data_availability_header.go:65-75
 *     -> rsmt2d v0.14.0 (EXT): Q0->Q1 rows, Q0->Q2 cols, Q2->Q3 rows
 *     (specs/src/specs/data_structures.md:306-310).
 *   - Leopard RS encode, klauspost/reedsolomon v1.12.1 (EXT, not vendored):
 *     leopard8.go initLUTs8/initFFT8/ifftDITEncoder8/fftDIT8 and leopard.go
 *     (GF(2^16)) -- restated from the published algorithm.
 *   - NMT leaf/node hashing: test/util/malicious/hasher.go:186-310 (in-tree copy
 *     of nmt v0.22.0 NmtHasher), namespace prefixing + quadrant test
 *     pkg/wrapper/nmt_wrapper.go:93-140, IgnoreMaxNamespace(true).
 *   - Push-order check: nmt validateAndExtractNamespace (ErrInvalidPushOrder).
 *   - Data root: pkg/da/data_availability_header.go:92-108 ->
 *     go-square/merkle HashFromByteSlices (RFC-6962).
 *   - Synthetic input: SURVEY.md 8(d), mirrors test/util/testfactory/common.go:36-46.
 *
 * Two implementations of the same function live here:
 *   oracle_extend / oracle_roots      -- scalar, single thread, the checker;
 *   oracle_cpu_baseline               -- multi-threaded, same rsmt2d structure
 *                                         (every cell hashed once per axis), used
 *                                         only as bench.py's CPU baseline and
 *                                         tested bit-equal to the scalar path.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SHARE 512
#define NS 29
#define NODE 90

/* ------------------------------------------------------------------ */
/* SHA-256 (FIPS 180-4)                                                 */
/* ------------------------------------------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t st[8], const uint8_t *p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* SHA-NI compression (x86 SHA extensions), used by the CPU-baseline path when
 * the host supports it -- Go's crypto/sha256 does the same on amd64.  Tested
 * bit-equal to sha256_block (tests/test_oracle.py). */
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("sha,sse4.1,ssse3"))) static void sha256_block_ni(uint32_t st[8], const uint8_t *p) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i TMP = _mm_loadu_si128((const __m128i *)&st[0]);
    __m128i STATE1 = _mm_loadu_si128((const __m128i *)&st[4]);
    TMP = _mm_shuffle_epi32(TMP, 0xB1);          /* CDAB */
    STATE1 = _mm_shuffle_epi32(STATE1, 0x1B);    /* EFGH */
    __m128i STATE0 = _mm_alignr_epi8(TMP, STATE1, 8);   /* ABEF */
    STATE1 = _mm_blend_epi16(STATE1, TMP, 0xF0);        /* CDGH */
    const __m128i ABEF_SAVE = STATE0, CDGH_SAVE = STATE1;
    __m128i MSG, MSG0, MSG1, MSG2, MSG3;
    MSG0 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 0)), MASK);
    MSG1 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16)), MASK);
    MSG2 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 32)), MASK);
    MSG3 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 48)), MASK);
    __m128i W[4] = {MSG0, MSG1, MSG2, MSG3};
    for (int r = 0; r < 16; r++) {
        __m128i k = _mm_loadu_si128((const __m128i *)&K256[4 * r]);
        MSG = _mm_add_epi32(W[r & 3], k);
        STATE1 = _mm_sha256rnds2_epu32(STATE1, STATE0, MSG);
        MSG = _mm_shuffle_epi32(MSG, 0x0E);
        STATE0 = _mm_sha256rnds2_epu32(STATE0, STATE1, MSG);
        if (r < 12) {
            /* W[r+4] = msg2(msg1(W[r], W[r+1]) + alignr(W[r+3], W[r+2]), W[r+3]) */
            __m128i t = _mm_sha256msg1_epu32(W[r & 3], W[(r + 1) & 3]);
            t = _mm_add_epi32(t, _mm_alignr_epi8(W[(r + 3) & 3], W[(r + 2) & 3], 4));
            W[r & 3] = _mm_sha256msg2_epu32(t, W[(r + 3) & 3]);
        }
    }
    STATE0 = _mm_add_epi32(STATE0, ABEF_SAVE);
    STATE1 = _mm_add_epi32(STATE1, CDGH_SAVE);
    TMP = _mm_shuffle_epi32(STATE0, 0x1B);       /* FEBA */
    STATE1 = _mm_shuffle_epi32(STATE1, 0xB1);    /* DCHG */
    STATE0 = _mm_blend_epi16(TMP, STATE1, 0xF0); /* DCBA */
    STATE1 = _mm_alignr_epi8(STATE1, TMP, 8);    /* ABEF */
    _mm_storeu_si128((__m128i *)&st[0], STATE0);
    _mm_storeu_si128((__m128i *)&st[4], STATE1);
}
static int have_sha_ni(void) {
    static int v = -1;
    if (v < 0) v = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
    return v;
}
#else
static void sha256_block_ni(uint32_t st[8], const uint8_t *p) { sha256_block(st, p); }
static int have_sha_ni(void) { return 0; }
#endif

/* 0 = portable scalar (the checker), 1 = SHA-NI when available (baseline). */
static __thread int g_fast = 0;
static void sha_block_dispatch(uint32_t st[8], const uint8_t *p) {
    if (g_fast && have_sha_ni()) sha256_block_ni(st, p);
    else sha256_block(st, p);
}

void oracle_sha256_block_test(uint32_t st[8], const uint8_t *p, int ni) {
    if (ni && have_sha_ni()) sha256_block_ni(st, p);
    else sha256_block(st, p);
}
int oracle_have_sha_ni(void) { return have_sha_ni(); }

typedef struct { uint32_t st[8]; uint8_t buf[64]; uint64_t len; } sha_ctx;

static void sha_init(sha_ctx *c) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(c->st, iv, sizeof iv);
    c->len = 0;
}
static void sha_update(sha_ctx *c, const uint8_t *p, size_t n) {
    while (n) {
        size_t off = c->len & 63, take = 64 - off;
        if (take > n) take = n;
        memcpy(c->buf + off, p, take);
        c->len += take; p += take; n -= take;
        if ((c->len & 63) == 0) sha_block_dispatch(c->st, c->buf);
    }
}
static void sha_final(sha_ctx *c, uint8_t out[32]) {
    uint64_t bits = c->len * 8;
    uint8_t pad = 0x80, z = 0;
    sha_update(c, &pad, 1);
    while ((c->len & 63) != 56) sha_update(c, &z, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha_update(c, l, 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = c->st[i] >> 24; out[4 * i + 1] = c->st[i] >> 16;
        out[4 * i + 2] = c->st[i] >> 8; out[4 * i + 3] = c->st[i];
    }
}

void oracle_sha256(const uint8_t *p, size_t n, uint8_t out[32]) {
    sha_ctx c; sha_init(&c); sha_update(&c, p, n); sha_final(&c, out);
}

/* ------------------------------------------------------------------ */
/* Leopard fields                                                       */
/* ------------------------------------------------------------------ */
typedef struct {
    int bits;
    uint32_t order, mod;
    uint16_t *log, *exp, *skew;
} field;

static field F8, F16;
static pthread_once_t fields_once = PTHREAD_ONCE_INIT;

static uint32_t add_mod(const field *F, uint32_t a, uint32_t b) {
    uint32_t s = a + b;
    return (s + (s >> F->bits)) & F->mod;
}
static uint32_t mul_log(const field *F, uint32_t a, uint32_t log_b) {
    return a == 0 ? 0 : F->exp[add_mod(F, F->log[a], log_b)];
}

static void field_init(field *F, int bits, uint32_t poly, const uint16_t *cantor) {
    F->bits = bits; F->order = 1u << bits; F->mod = F->order - 1;
    F->log = calloc(F->order, 2); F->exp = calloc(F->order, 2); F->skew = calloc(F->mod, 2);
    uint32_t state = 1;
    for (uint32_t i = 0; i < F->mod; i++) {      /* initLUTs: LFSR */
        F->exp[state] = (uint16_t)i;
        state <<= 1;
        if (state >= F->order) state ^= poly;
    }
    F->exp[0] = (uint16_t)F->mod;
    F->log[0] = 0;                               /* Cantor basis conversion */
    for (int i = 0; i < bits; i++) {
        uint32_t width = 1u << i;
        for (uint32_t j = 0; j < width; j++) F->log[j + width] = F->log[j] ^ cantor[i];
    }
    for (uint32_t i = 0; i < F->order; i++) F->log[i] = F->exp[F->log[i]];
    for (uint32_t i = 0; i < F->order; i++) F->exp[F->log[i]] = (uint16_t)i;
    F->exp[F->mod] = F->exp[0];

    uint32_t temp[16];                           /* initFFT: skew */
    for (int i = 1; i < bits; i++) temp[i - 1] = 1u << i;
    for (int m = 0; m < bits - 1; m++) {
        uint32_t step = 1u << (m + 1);
        F->skew[(1u << m) - 1] = 0;
        for (int i = m; i < bits - 1; i++) {
            uint32_t s = 1u << (i + 1);
            for (uint32_t j = (1u << m) - 1; j < s; j += step) F->skew[j + s] = F->skew[j] ^ temp[i];
        }
        temp[m] = F->mod - F->log[mul_log(F, temp[m], F->log[temp[m] ^ 1])];
        for (int i = m + 1; i < bits - 1; i++)
            temp[i] = mul_log(F, temp[i], add_mod(F, F->log[temp[i] ^ 1], temp[m]));
    }
    for (uint32_t i = 0; i < F->mod; i++) F->skew[i] = F->log[F->skew[i]];
}

static void fields_init(void) {
    static const uint16_t c8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
    static const uint16_t c16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                     0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
    field_init(&F8, 8, 0x11D, c8);
    field_init(&F16, 16, 0x1002D, c16);
}

/* Exposed for tests / kernel table generation cross-checks. */
const uint16_t *oracle_table(int bits, int which) {
    pthread_once(&fields_once, fields_init);
    field *F = bits == 8 ? &F8 : &F16;
    return which == 0 ? F->log : which == 1 ? F->exp : F->skew;
}

/* Encode one codeword of m symbols per lane, `lanes` lanes, symbols stored
 * w[i*lanes + lane].  Radix-2 restatement of ifftDITEncoder + fftDIT. */
static void encode_symbols(const field *F, uint16_t *w, uint32_t m, size_t lanes) {
    for (uint32_t d = 1; d < m; d <<= 1)
        for (uint32_t g = 0; g < m; g += 2 * d) {
            uint32_t L = F->skew[m - 1 + g + d];
            for (uint32_t i = g; i < g + d; i++) {
                uint16_t *x = w + (size_t)i * lanes, *y = w + (size_t)(i + d) * lanes;
                for (size_t l = 0; l < lanes; l++) {
                    y[l] ^= x[l];
                    if (L != F->mod) x[l] ^= mul_log(F, y[l], L);
                }
            }
        }
    for (uint32_t d = m >> 1; d >= 1; d >>= 1)
        for (uint32_t g = 0; g < m; g += 2 * d) {
            uint32_t L = F->skew[g + d - 1];
            for (uint32_t i = g; i < g + d; i++) {
                uint16_t *x = w + (size_t)i * lanes, *y = w + (size_t)(i + d) * lanes;
                for (size_t l = 0; l < lanes; l++) {
                    if (L != F->mod) x[l] ^= mul_log(F, y[l], L);
                    y[l] ^= x[l];
                }
            }
        }
}

/* ------------------------------------------------------------------ */
/* CPU-baseline RS: same butterflies, multiply with PSHUFB nibble tables */
/* (the klauspost/reedsolomon amd64 technique: mulAdd via VPSHUFB).     */
/* Used only by oracle_cpu_baseline; tested bit-equal to the scalar path. */
/* ------------------------------------------------------------------ */
#if defined(__x86_64__)
__attribute__((target("avx2"))) static void mul_add8_avx2(uint8_t *x, const uint8_t *y, size_t n, const field *F,
                                                           uint32_t L) {
    uint8_t tl[16], th[16];
    for (int i = 0; i < 16; i++) { tl[i] = (uint8_t)mul_log(F, i, L); th[i] = (uint8_t)mul_log(F, i << 4, L); }
    const __m256i TL = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)tl));
    const __m256i TH = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)th));
    const __m256i M = _mm256_set1_epi8(0x0F);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i v = _mm256_loadu_si256((const __m256i *)(y + i));
        __m256i lo = _mm256_and_si256(v, M), hi = _mm256_and_si256(_mm256_srli_epi64(v, 4), M);
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(TL, lo), _mm256_shuffle_epi8(TH, hi));
        _mm256_storeu_si256((__m256i *)(x + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(x + i)), p));
    }
    for (; i < n; i++) x[i] ^= (uint8_t)mul_log(F, y[i], L);
}
/* GF(2^16), lo/hi split layout: per 64-byte block b[0..31] lo, b[32..63] hi. */
__attribute__((target("avx2"))) static void mul_add16_avx2(uint8_t *x, const uint8_t *y, size_t n, const field *F,
                                                            uint32_t L) {
    uint8_t t[8][16];   /* [nibble q][lo/hi out][16] */
    for (int q = 0; q < 4; q++)
        for (int v = 0; v < 16; v++) {
            uint32_t pr = mul_log(F, (uint32_t)v << (4 * q), L);
            t[2 * q][v] = (uint8_t)pr;
            t[2 * q + 1][v] = (uint8_t)(pr >> 8);
        }
    __m256i T[8];
    for (int i = 0; i < 8; i++) T[i] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[i]));
    const __m256i M = _mm256_set1_epi8(0x0F);
    for (size_t i = 0; i + 64 <= n; i += 64) {
        __m256i lo = _mm256_loadu_si256((const __m256i *)(y + i)), hi = _mm256_loadu_si256((const __m256i *)(y + i + 32));
        __m256i n0 = _mm256_and_si256(lo, M), n1 = _mm256_and_si256(_mm256_srli_epi64(lo, 4), M);
        __m256i n2 = _mm256_and_si256(hi, M), n3 = _mm256_and_si256(_mm256_srli_epi64(hi, 4), M);
        __m256i pl = _mm256_xor_si256(_mm256_xor_si256(_mm256_shuffle_epi8(T[0], n0), _mm256_shuffle_epi8(T[2], n1)),
                                      _mm256_xor_si256(_mm256_shuffle_epi8(T[4], n2), _mm256_shuffle_epi8(T[6], n3)));
        __m256i ph = _mm256_xor_si256(_mm256_xor_si256(_mm256_shuffle_epi8(T[1], n0), _mm256_shuffle_epi8(T[3], n1)),
                                      _mm256_xor_si256(_mm256_shuffle_epi8(T[5], n2), _mm256_shuffle_epi8(T[7], n3)));
        _mm256_storeu_si256((__m256i *)(x + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(x + i)), pl));
        _mm256_storeu_si256((__m256i *)(x + i + 32),
                            _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(x + i + 32)), ph));
    }
}
__attribute__((target("avx2"))) static void xor_avx2(uint8_t *y, const uint8_t *x, size_t n) {
    size_t i = 0;
    for (; i + 32 <= n; i += 32)
        _mm256_storeu_si256((__m256i *)(y + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(y + i)),
                                                                  _mm256_loadu_si256((const __m256i *)(x + i))));
    for (; i < n; i++) y[i] ^= x[i];
}
static int have_avx2(void) {
    static int v = -1;
    if (v < 0) v = __builtin_cpu_supports("avx2");
    return v;
}
#else
static int have_avx2(void) { return 0; }
static void mul_add8_avx2(uint8_t *x, const uint8_t *y, size_t n, const field *F, uint32_t L) {}
static void mul_add16_avx2(uint8_t *x, const uint8_t *y, size_t n, const field *F, uint32_t L) {}
static void xor_avx2(uint8_t *y, const uint8_t *x, size_t n) {}
#endif

/* Leopard encode on byte shards w[i] (len bytes each), in place: w[0..k) data
 * -> parity.  Same layer order as encode_symbols. */
static void encode_bytes_fast(const field *F, uint8_t **w, uint32_t m, size_t len) {
    const int f16 = F->bits == 16;
    for (uint32_t d = 1; d < m; d <<= 1)
        for (uint32_t g = 0; g < m; g += 2 * d) {
            uint32_t L = F->skew[m - 1 + g + d];
            for (uint32_t i = g; i < g + d; i++) {
                xor_avx2(w[i + d], w[i], len);
                if (L != F->mod) (f16 ? mul_add16_avx2 : mul_add8_avx2)(w[i], w[i + d], len, F, L);
            }
        }
    for (uint32_t d = m >> 1; d >= 1; d >>= 1)
        for (uint32_t g = 0; g < m; g += 2 * d) {
            uint32_t L = F->skew[g + d - 1];
            for (uint32_t i = g; i < g + d; i++) {
                if (L != F->mod) (f16 ? mul_add16_avx2 : mul_add8_avx2)(w[i], w[i + d], len, F, L);
                xor_avx2(w[i + d], w[i], len);
            }
        }
}

/* LeoRSCodec.Encode on k shards of `len` bytes given as pointers (strided
 * access lets the caller encode a column in place).  Returns 0 or -2 for a
 * chunk size that is not a multiple of 64. */
int oracle_leopard_encode_ptrs(const uint8_t *const *data, uint8_t *const *parity, uint32_t k, uint32_t len) {
    pthread_once(&fields_once, fields_init);
    if (len % 64) return -2;
    if (k == 1) { memcpy(parity[0], data[0], len); return 0; }
    const field *F = (2 * k <= 256) ? &F8 : &F16;
    if (g_fast && have_avx2()) {     /* CPU-baseline path: work in place in the parity shards */
        uint8_t **w = malloc(k * sizeof *w);
        for (uint32_t i = 0; i < k; i++) { memcpy(parity[i], data[i], len); w[i] = parity[i]; }
        encode_bytes_fast(F, w, k, len);
        free(w);
        return 0;
    }
    if (F->bits == 8) {
        uint16_t *w = malloc((size_t)k * len * 2);
        for (uint32_t i = 0; i < k; i++)
            for (uint32_t b = 0; b < len; b++) w[(size_t)i * len + b] = data[i][b];
        encode_symbols(F, w, k, len);
        for (uint32_t i = 0; i < k; i++)
            for (uint32_t b = 0; b < len; b++) parity[i][b] = (uint8_t)w[(size_t)i * len + b];
        free(w);
    } else {
        size_t lanes = len / 2;
        uint16_t *w = malloc((size_t)k * lanes * 2);
        for (uint32_t i = 0; i < k; i++)
            for (uint32_t blk = 0; blk < len / 64; blk++)
                for (int s = 0; s < 32; s++)
                    w[(size_t)i * lanes + blk * 32 + s] =
                        data[i][blk * 64 + s] | (uint16_t)data[i][blk * 64 + 32 + s] << 8;
        encode_symbols(F, w, k, lanes);
        for (uint32_t i = 0; i < k; i++)
            for (uint32_t blk = 0; blk < len / 64; blk++)
                for (int s = 0; s < 32; s++) {
                    uint16_t v = w[(size_t)i * lanes + blk * 32 + s];
                    parity[i][blk * 64 + s] = (uint8_t)v;
                    parity[i][blk * 64 + 32 + s] = (uint8_t)(v >> 8);
                }
        free(w);
    }
    return 0;
}

int oracle_leopard_encode(const uint8_t *data, uint8_t *parity, uint32_t k, uint32_t len) {
    const uint8_t **dp = malloc(k * sizeof *dp);
    uint8_t **pp = malloc(k * sizeof *pp);
    for (uint32_t i = 0; i < k; i++) { dp[i] = data + (size_t)i * len; pp[i] = parity + (size_t)i * len; }
    int rc = oracle_leopard_encode_ptrs(dp, pp, k, len);
    free(dp); free(pp);
    return rc;
}

/* ------------------------------------------------------------------ */
/* EDS                                                                  */
/* ------------------------------------------------------------------ */
#define CELL(eds, W, r, c) ((eds) + ((size_t)(r) * (W) + (c)) * SHARE)

static void encode_axis(uint8_t *eds, uint32_t k, int col, uint32_t idx) {
    uint32_t W = 2 * k;
    const uint8_t **dp = malloc(k * sizeof *dp);
    uint8_t **pp = malloc(k * sizeof *pp);
    for (uint32_t i = 0; i < k; i++) {
        dp[i] = col ? CELL(eds, W, i, idx) : CELL(eds, W, idx, i);
        pp[i] = col ? CELL(eds, W, k + i, idx) : CELL(eds, W, idx, k + i);
    }
    oracle_leopard_encode_ptrs(dp, pp, k, SHARE);
    free(dp); free(pp);
}

/* ods: k*k*512 row-major; eds: (2k)^2*512 row-major. */
int oracle_extend(const uint8_t *ods, uint32_t k, uint8_t *eds) {
    if (k == 0 || (k & (k - 1))) return -1;
    uint32_t W = 2 * k;
    for (uint32_t r = 0; r < k; r++) memcpy(CELL(eds, W, r, 0), ods + (size_t)r * k * SHARE, (size_t)k * SHARE);
    for (uint32_t i = 0; i < k; i++) encode_axis(eds, k, 0, i);     /* Q0 -> Q1 */
    for (uint32_t i = 0; i < k; i++) encode_axis(eds, k, 1, i);     /* Q0 -> Q2 */
    for (uint32_t i = k; i < W; i++) encode_axis(eds, k, 0, i);     /* Q2 -> Q3 */
    return 0;
}

/* ------------------------------------------------------------------ */
/* NMT                                                                  */
/* ------------------------------------------------------------------ */
static const uint8_t PARITY_NS[NS] = {
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};

void oracle_hash_leaf(const uint8_t ns[NS], const uint8_t *share, uint8_t out[NODE]) {
    sha_ctx c; uint8_t pre = 0;
    sha_init(&c);
    sha_update(&c, &pre, 1);
    sha_update(&c, ns, NS);
    sha_update(&c, share, SHARE);
    memcpy(out, ns, NS); memcpy(out + NS, ns, NS);
    sha_final(&c, out + 2 * NS);
}

void oracle_hash_node(const uint8_t l[NODE], const uint8_t r[NODE], uint8_t out[NODE]) {
    uint8_t tmp[NODE];
    sha_ctx c; uint8_t pre = 1;
    sha_init(&c);
    sha_update(&c, &pre, 1);
    sha_update(&c, l, NODE);
    sha_update(&c, r, NODE);
    memcpy(tmp, l, NS);
    memcpy(tmp + NS, memcmp(r, PARITY_NS, NS) == 0 ? l + NS : r + NS, NS);
    sha_final(&c, tmp + 2 * NS);
    memcpy(out, tmp, NODE);
}

/* Root of one row (col=0) or column (col=1): W leaves, W a power of two.
 * Returns 0, or -3 on namespace push-order violation (nmt ErrInvalidPushOrder);
 * on error *bad_pos receives the index of the offending push. */
static int axis_root(const uint8_t *eds, uint32_t k, int col, uint32_t idx, uint8_t out[NODE], uint32_t *bad_pos) {
    uint32_t W = 2 * k;
    uint8_t *nodes = malloc((size_t)W * NODE);
    const uint8_t *last = NULL;
    for (uint32_t j = 0; j < W; j++) {
        const uint8_t *cell = col ? CELL(eds, W, j, idx) : CELL(eds, W, idx, j);
        const uint8_t *ns = (j < k && idx < k) ? cell : PARITY_NS;
        if (last && memcmp(ns, last, NS) < 0) { free(nodes); if (bad_pos) *bad_pos = j; return -3; }
        last = ns;
        oracle_hash_leaf(ns, cell, nodes + (size_t)j * NODE);
    }
    for (uint32_t n = W; n > 1; n >>= 1)
        for (uint32_t i = 0; i < n / 2; i++)
            oracle_hash_node(nodes + (size_t)(2 * i) * NODE, nodes + (size_t)(2 * i + 1) * NODE, nodes + (size_t)i * NODE);
    memcpy(out, nodes, NODE);
    free(nodes);
    return 0;
}

/* rsmt2d RowRoots then ColRoots. Returns 0 or -3 (push order). err_axis/err_idx
 * report the first failing tree (rows scanned before columns). */
int oracle_roots(const uint8_t *eds, uint32_t k, uint8_t *rows, uint8_t *cols, int *err_axis, uint32_t *err_idx) {
    uint32_t W = 2 * k;
    for (int ax = 0; ax < 2; ax++)
        for (uint32_t i = 0; i < W; i++) {
            uint32_t pos;
            if (axis_root(eds, k, ax, i, (ax ? cols : rows) + (size_t)i * NODE, &pos)) {
                if (err_axis) *err_axis = ax;
                if (err_idx) *err_idx = i;
                return -3;
            }
        }
    return 0;
}

/* RFC-6962 over n items of `isz` bytes (go-square/merkle HashFromByteSlices). */
static void merkle(const uint8_t *items, size_t n, size_t isz, uint8_t out[32]) {
    if (n == 0) { oracle_sha256(NULL, 0, out); return; }
    if (n == 1) {
        uint8_t *b = malloc(isz + 1);
        b[0] = 0; memcpy(b + 1, items, isz);
        oracle_sha256(b, isz + 1, out);
        free(b);
        return;
    }
    size_t s = 1;
    while (s * 2 < n) s *= 2;
    uint8_t b[65];
    b[0] = 1;
    merkle(items, s, isz, b + 1);
    merkle(items + s * isz, n - s, isz, b + 33);
    oracle_sha256(b, 65, out);
}

void oracle_data_root(const uint8_t *rows, const uint8_t *cols, uint32_t W, uint8_t out[32]) {
    uint8_t *all = malloc((size_t)2 * W * NODE + 1);
    memcpy(all, rows, (size_t)W * NODE);
    memcpy(all + (size_t)W * NODE, cols, (size_t)W * NODE);
    merkle(all, (size_t)2 * W, NODE, out);
    free(all);
}

void oracle_merkle(const uint8_t *items, size_t n, size_t isz, uint8_t out[32]) { merkle(items, n, isz, out); }

int oracle_extend_dah(const uint8_t *ods, uint32_t k, uint8_t *eds, uint8_t *rows, uint8_t *cols, uint8_t root[32]) {
    int rc = oracle_extend(ods, k, eds);
    if (rc) return rc;
    rc = oracle_roots(eds, k, rows, cols, NULL, NULL);
    if (rc) return rc;
    oracle_data_root(rows, cols, 2 * k, root);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Synthetic random-namespace square                    */
/* ------------------------------------------------------------------ */
typedef struct { uint64_t state; uint8_t buf[8]; int avail; } smix;
static uint8_t smix_byte(smix *s) {
    if (!s->avail) {
        s->state += 0x9E3779B97F4A7C15ull;
        uint64_t z = s->state;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (int i = 0; i < 8; i++) s->buf[i] = (uint8_t)(z >> (8 * i));
        s->avail = 8;
    }
    return s->buf[8 - s->avail--];
}
static int cmp_share(const void *a, const void *b) { return memcmp(a, b, SHARE); }

void oracle_random_square(uint32_t k, uint64_t square_index, uint8_t *ods) {
    smix s = {0xCE1E57A0ull + square_index, {0}, 0};
    size_t n = (size_t)k * k;
    for (size_t i = 0; i < n; i++) {
        uint8_t *sh = ods + i * SHARE;
        memset(sh, 0, 19);
        for (;;) {
            int nz = 0;
            for (int b = 0; b < 10; b++) { sh[19 + b] = smix_byte(&s); if (b < 9) nz |= sh[19 + b]; }
            if (nz) break;
        }
        for (int b = NS; b < SHARE; b++) sh[b] = smix_byte(&s);
    }
    qsort(ods, n, SHARE, cmp_share);
}

/* ------------------------------------------------------------------ */
/* CPU baseline: rsmt2d structure, multi-threaded                       */
/* ------------------------------------------------------------------ */
typedef struct {
    uint8_t *eds; uint32_t k; int phase; uint32_t next; pthread_mutex_t mu;
    uint8_t *rows, *cols; int err;
} job;

static void *worker(void *arg) {
    job *j = arg;
    g_fast = 1;   /* SHA-NI + AVX2 nibble-table RS, like Go's amd64 assembly */
    uint32_t W = 2 * j->k;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t t = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (j->phase == 0) {            /* rows + cols of Q0, interleaved like errgroup */
            if (t >= 2 * j->k) break;
            encode_axis(j->eds, j->k, t & 1, t >> 1);
        } else if (j->phase == 1) {     /* Q2 -> Q3 rows */
            if (t >= j->k) break;
            encode_axis(j->eds, j->k, 0, j->k + t);
        } else {                        /* roots: one tree per task, each cell hashed per axis */
            if (t >= 2 * W) break;
            int ax = t & 1; uint32_t i = t >> 1;
            if (axis_root(j->eds, j->k, ax, i, (ax ? j->cols : j->rows) + (size_t)i * NODE, NULL)) j->err = -3;
        }
    }
    return NULL;
}

static void run_phase(job *j, int phase, int nthreads) {
    j->phase = phase; j->next = 0;
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, worker, j);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
}

int oracle_cpu_baseline(const uint8_t *ods, uint32_t k, uint8_t *eds, uint8_t *rows, uint8_t *cols,
                        uint8_t root[32], int nthreads) {
    if (nthreads == 0) {   /* scalar single-thread path through the same scheduler (tests) */
        return oracle_extend_dah(ods, k, eds, rows, cols, root);
    }
    pthread_once(&fields_once, fields_init);
    if (k == 0 || (k & (k - 1))) return -1;
    if (nthreads < 1) nthreads = 1;
    uint32_t W = 2 * k;
    for (uint32_t r = 0; r < k; r++) memcpy(CELL(eds, W, r, 0), ods + (size_t)r * k * SHARE, (size_t)k * SHARE);
    job j = {eds, k, 0, 0, PTHREAD_MUTEX_INITIALIZER, rows, cols, 0};
    run_phase(&j, 0, nthreads);
    run_phase(&j, 1, nthreads);
    run_phase(&j, 2, nthreads);
    if (j.err) return j.err;
    oracle_data_root(rows, cols, W, root);
    return 0;
}
