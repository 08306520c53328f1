/*
 * rs_oracle.c -- CPU restatement of github.com/klauspost/reedsolomon
 *                @ v0.0.0-20180704173009-925cb01d6510 (pinned by the reference at
 *                /root/reference/go.mod:20, go.sum:33-34).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP engine in
 * blb_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product path (blb_amd/) never links or calls it.
 *
 * The klauspost module is not vendored in the reference tree and no Go toolchain exists
 * in this image, so this is a restatement of the module's published algorithm (see
 * SURVEY.md Appendix A), anchored on blb's call sites:
 *   - reedsolomon.New          internal/tractserver/store.go:1022, client/blb/reconstruct.go:166
 *   - Encoder.Encode           internal/tractserver/store.go:1099
 *   - Encoder.Reconstruct      internal/tractserver/store.go:1133
 *   - Encoder.Verify           internal/tractserver/store.go:1136
 *   - Encoder.ReconstructData  client/blb/reconstruct.go:173
 *
 * Pinning: the reference tree holds no golden RS vectors (its tests only round-trip via
 * Verify: internal/tractserver/store_test.go:810-814,875-878).  The restatement is pinned
 * by the dependency's own published known-answer tests (tests/golden/published_kat.json,
 * tests/test_published_kat.py): TestOneEncode's fixed RS(5,5) parity bytes, TestGalois'
 * galMultiply/galExp values, TestMatrixMultiply and TestMatrixInverse[2]; CRC-32C by Go's
 * hash/crc32 Castagnoli golden table.  It is further cross-checked against an independent
 * numpy restatement (oracle/rs_numpy.py, carry-less multiplication instead of log/exp
 * tables), the Backblaze/klauspost RS(4,2) matrix and algebraic properties.  No output of
 * the reference itself exists here (Go and the module are absent).
 *
 * Two compute paths, same results:
 *   rso_code_scalar   -- klauspost's pure-Go path: galMulSlice/galMulSliceXor over mulTable
 *   rso_code_avx2     -- klauspost's galMulAVX2[Xor] path: 16-entry low/high nibble tables
 *                        applied with vpshufb; used as the cpu_baseline ("port") in bench.py,
 *                        split over OpenMP threads the way codeSomeShardsP splits byte
 *                        ranges over goroutines.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* klauspost error values (reedsolomon.go), as negative codes. */
enum {
    RSO_OK = 0,
    RSO_ERR_INV_SHARD_NUM = -1,   /* ErrInvShardNum  */
    RSO_ERR_MAX_SHARD_NUM = -2,   /* ErrMaxShardNum  */
    RSO_ERR_TOO_FEW_SHARDS = -3,  /* ErrTooFewShards */
    RSO_ERR_SHARD_NO_DATA = -4,   /* ErrShardNoData  */
    RSO_ERR_SHARD_SIZE = -5,      /* ErrShardSize    */
    RSO_ERR_SINGULAR = -6,        /* errSingular (matrix.go) */
    RSO_ERR_ALLOC = -7,
};

/* ---- galois.go: GF(2^8), generating polynomial 29 (x^8+x^4+x^3+x^2+1), alpha = 2 ---- */
static uint8_t exp_table[510];
static uint8_t log_table[256];
static uint8_t mul_table[256][256];
static uint8_t mul_low[256][16];   /* galois.go mulTableLow  : c * i        */
static uint8_t mul_high[256][16];  /* galois.go mulTableHigh : c * (i << 4) */
static int tables_ready = 0;

static void init_tables(void) {
    if (tables_ready) return;
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        exp_table[i] = (uint8_t)x;
        exp_table[i + 255] = (uint8_t)x;
        log_table[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11d;
    }
    log_table[0] = 0; /* unused (galMultiply special-cases zero) */
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            mul_table[a][b] = (a == 0 || b == 0) ? 0
                              : exp_table[log_table[a] + log_table[b]];
    for (int c = 0; c < 256; c++)
        for (int i = 0; i < 16; i++) {
            mul_low[c][i] = mul_table[c][i];
            mul_high[c][i] = mul_table[c][i << 4];
        }
    tables_ready = 1;
}

uint8_t rso_gal_mul(uint8_t a, uint8_t b) { init_tables(); return mul_table[a][b]; }

/* galois.go galExp(a, n): 1 if n==0, 0 if a==0, else exp[(log a * n) mod 255]. */
uint8_t rso_gal_exp(uint8_t a, int n) {
    init_tables();
    if (n == 0) return 1;
    if (a == 0) return 0;
    int r = (int)log_table[a] * n;
    while (r >= 255) r -= 255;
    return exp_table[r];
}

static uint8_t gal_div(uint8_t a, uint8_t b) {
    if (a == 0) return 0;
    int r = (int)log_table[a] - (int)log_table[b];
    if (r < 0) r += 255;
    return exp_table[r];
}

/* ---- matrix.go: row-major rows x cols byte matrices ---- */

/* matrix.go vandermonde(rows, cols): V[r][c] = galExp(byte(r), c). */
static void vandermonde(int rows, int cols, uint8_t* v) {
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) v[r * cols + c] = rso_gal_exp((uint8_t)r, c);
}

/* matrix.go Multiply: (ar x ac) * (ac x bc). */
static void mat_mul(const uint8_t* a, int ar, int ac, const uint8_t* b, int bc, uint8_t* out) {
    for (int r = 0; r < ar; r++)
        for (int c = 0; c < bc; c++) {
            uint8_t v = 0;
            for (int i = 0; i < ac; i++) v ^= mul_table[a[r * ac + i]][b[i * bc + c]];
            out[r * bc + c] = v;
        }
}

/* matrix.go Invert: Gauss-Jordan on [A | I] with row swaps (gaussianElimination). */
int rso_invert(int n, const uint8_t* in, uint8_t* out) {
    init_tables();
    int w = 2 * n;
    uint8_t* aug = (uint8_t*)malloc((size_t)n * w);
    if (!aug) return RSO_ERR_ALLOC;
    for (int r = 0; r < n; r++) {
        memcpy(aug + r * w, in + r * n, n);
        memset(aug + r * w + n, 0, n);
        aug[r * w + n + r] = 1;
    }
    for (int r = 0; r < n; r++) {
        if (aug[r * w + r] == 0) {
            for (int below = r + 1; below < n; below++)
                if (aug[below * w + r] != 0) {
                    for (int j = 0; j < w; j++) {
                        uint8_t t = aug[r * w + j];
                        aug[r * w + j] = aug[below * w + j];
                        aug[below * w + j] = t;
                    }
                    break;
                }
        }
        if (aug[r * w + r] == 0) { free(aug); return RSO_ERR_SINGULAR; }
        if (aug[r * w + r] != 1) {
            uint8_t scale = gal_div(1, aug[r * w + r]);
            for (int j = 0; j < w; j++) aug[r * w + j] = mul_table[aug[r * w + j]][scale];
        }
        for (int below = r + 1; below < n; below++) {
            uint8_t s = aug[below * w + r];
            if (s) for (int j = 0; j < w; j++) aug[below * w + j] ^= mul_table[s][aug[r * w + j]];
        }
    }
    for (int d = 0; d < n; d++)
        for (int above = 0; above < d; above++) {
            uint8_t s = aug[above * w + d];
            if (s) for (int j = 0; j < w; j++) aug[above * w + j] ^= mul_table[s][aug[d * w + j]];
        }
    for (int r = 0; r < n; r++) memcpy(out + r * n, aug + r * w + n, n);
    free(aug);
    return RSO_OK;
}

/* reedsolomon.go New() argument checks + buildMatrix(): M = V * inv(V[0:k]).
 * out must hold (k+m)*k bytes. */
int rso_build_matrix(int k, int m, uint8_t* out) {
    init_tables();
    if (k <= 0 || m <= 0) return RSO_ERR_INV_SHARD_NUM;
    if (k + m > 256) return RSO_ERR_MAX_SHARD_NUM;
    int n = k + m;
    uint8_t* v = (uint8_t*)malloc((size_t)n * k);
    uint8_t* top_inv = (uint8_t*)malloc((size_t)k * k);
    if (!v || !top_inv) { free(v); free(top_inv); return RSO_ERR_ALLOC; }
    vandermonde(n, k, v);
    int rc = rso_invert(k, v, top_inv); /* top = V[0:k][0:k] = first k rows */
    if (rc == RSO_OK) mat_mul(v, n, k, top_inv, k, out);
    free(v); free(top_inv);
    return rc;
}

/* ---- galMulSlice / galMulSliceXor (pure-Go mulTable path) ---- */
static void gal_mul_slice(uint8_t c, const uint8_t* in, uint8_t* out, size_t n, int xor_) {
    const uint8_t* mt = mul_table[c];
    if (xor_) for (size_t i = 0; i < n; i++) out[i] ^= mt[in[i]];
    else      for (size_t i = 0; i < n; i++) out[i] = mt[in[i]];
}

#if defined(__x86_64__)
/* galois_amd64.s galMulAVX2 / galMulAVX2Xor: per 32 bytes,
 *   lo = in & 0x0f; hi = (in >> 4) & 0x0f;
 *   out (^)= vpshufb(low[c], lo) ^ vpshufb(high[c], hi)                       */
__attribute__((target("avx2")))
static void gal_mul_slice_avx2(uint8_t c, const uint8_t* in, uint8_t* out, size_t n, int xor_) {
    __m128i l128 = _mm_loadu_si128((const __m128i*)mul_low[c]);
    __m128i h128 = _mm_loadu_si128((const __m128i*)mul_high[c]);
    __m256i lo_t = _mm256_broadcastsi128_si256(l128);
    __m256i hi_t = _mm256_broadcastsi128_si256(h128);
    __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i*)(in + i));
        __m256i lo = _mm256_and_si256(x, mask);
        __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(lo_t, lo), _mm256_shuffle_epi8(hi_t, hi));
        if (xor_) p = _mm256_xor_si256(p, _mm256_loadu_si256((const __m256i*)(out + i)));
        _mm256_storeu_si256((__m256i*)(out + i), p);
    }
    /* klauspost handles the < 32-byte remainder with the pure-Go loop */
    gal_mul_slice(c, in + i, out + i, n - i, xor_);
}
static int have_avx2(void) { return __builtin_cpu_supports("avx2"); }
#else
static int have_avx2(void) { return 0; }
#endif

/* reedsolomon.go codeSomeShards: for c in inputs, for each output row: mul(c==0)/mulXor. */
static void code_some_shards(const uint8_t* rows, int in_count, int out_count,
                             const uint8_t* const* inputs, uint8_t* const* outputs,
                             size_t off, size_t n, int use_avx2) {
    for (int c = 0; c < in_count; c++)
        for (int r = 0; r < out_count; r++) {
            uint8_t coef = rows[r * in_count + c];
#if defined(__x86_64__)
            if (use_avx2) { gal_mul_slice_avx2(coef, inputs[c] + off, outputs[r] + off, n, c != 0); continue; }
#endif
            gal_mul_slice(coef, inputs[c] + off, outputs[r] + off, n, c != 0);
        }
}

/* rows: out_count x in_count coefficient matrix.  threads > 1 splits the byte range like
 * codeSomeShardsP (goroutines over contiguous column ranges).  Results are independent of
 * the split because byte columns are independent. */
void rso_code(const uint8_t* rows, int in_count, int out_count,
              const uint8_t* const* inputs, uint8_t* const* outputs, size_t n,
              int use_avx2, int threads) {
    init_tables();
    use_avx2 = use_avx2 && have_avx2();
    if (threads <= 1 || n < 4096) {
        code_some_shards(rows, in_count, out_count, inputs, outputs, 0, n, use_avx2);
        return;
    }
#ifdef _OPENMP
    size_t per = (n + (size_t)threads - 1) / (size_t)threads;
    per = (per + 63) & ~(size_t)63;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int t = 0; t < threads; t++) {
        size_t start = (size_t)t * per;
        if (start < n) {
            size_t len = (start + per > n) ? n - start : per;
            code_some_shards(rows, in_count, out_count, inputs, outputs, start, len, use_avx2);
        }
    }
#else
    code_some_shards(rows, in_count, out_count, inputs, outputs, 0, n, use_avx2);
#endif
}

int rso_have_avx2(void) { return have_avx2(); }
int rso_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* reedsolomon.go checkShards/shardSize: first non-zero length; nilok allows zero lengths. */
static int check_shards(int n, const size_t* lens, int nilok, size_t* size_out) {
    size_t size = 0;
    for (int i = 0; i < n; i++) if (lens[i]) { size = lens[i]; break; }
    if (size == 0) return RSO_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; i++)
        if (lens[i] != size && (lens[i] != 0 || !nilok)) return RSO_ERR_SHARD_SIZE;
    *size_out = size;
    return RSO_OK;
}

/* Encoder.Encode: shards[0..k) data in, shards[k..k+m) parity out (fully overwritten). */
int rso_encode(int k, int m, uint8_t* const* shards, const size_t* lens, int use_avx2, int threads) {
    uint8_t mat[256 * 256];
    int rc = rso_build_matrix(k, m, mat);
    if (rc) return rc;
    size_t size;
    if ((rc = check_shards(k + m, lens, 0, &size))) return rc;
    rso_code(mat + (size_t)k * k, k, m, (const uint8_t* const*)shards, shards + k, size, use_avx2, threads);
    return RSO_OK;
}

/* Encoder.Verify: recompute parity into temporaries and compare. *ok = 1 when equal. */
int rso_verify(int k, int m, const uint8_t* const* shards, const size_t* lens, int* ok) {
    uint8_t mat[256 * 256];
    int rc = rso_build_matrix(k, m, mat);
    if (rc) return rc;
    size_t size;
    if ((rc = check_shards(k + m, lens, 0, &size))) return rc;
    uint8_t** tmp = (uint8_t**)calloc((size_t)m, sizeof(uint8_t*));
    if (!tmp) return RSO_ERR_ALLOC;
    for (int i = 0; i < m; i++) {
        tmp[i] = (uint8_t*)malloc(size);
        if (!tmp[i]) { for (int j = 0; j < i; j++) free(tmp[j]); free(tmp); return RSO_ERR_ALLOC; }
    }
    rso_code(mat + (size_t)k * k, k, m, shards, tmp, size, 0, 1);
    *ok = 1;
    for (int i = 0; i < m; i++) if (memcmp(tmp[i], shards[k + i], size)) *ok = 0;
    for (int i = 0; i < m; i++) free(tmp[i]);
    free(tmp);
    return RSO_OK;
}

/* Encoder.reconstruct(shards, dataOnly).  lens[i]==0 marks a missing shard; its pointer
 * must address a buffer with room for the shard size (the "cap >= shardSize" reslice in
 * klauspost), or be NULL when the slot will not be produced (parity with data_only).
 * On return lens[] is updated for every slot that was produced.
 * The decode rows come from inv(M[valid]) with valid = first k present indices ascending. */
int rso_reconstruct(int k, int m, uint8_t* const* shards, size_t* lens, int data_only) {
    uint8_t mat[256 * 256];
    int rc = rso_build_matrix(k, m, mat);
    if (rc) return rc;
    int n = k + m;
    size_t size;
    if ((rc = check_shards(n, lens, 1, &size))) return rc;
    int present = 0;
    for (int i = 0; i < n; i++) present += lens[i] != 0;
    if (present == n) return RSO_OK;
    if (present < k) return RSO_ERR_TOO_FEW_SHARDS;

    int valid[256];
    const uint8_t* sub_shards[256];
    int sub = 0;
    for (int r = 0; r < n && sub < k; r++)
        if (lens[r]) { valid[sub] = r; sub_shards[sub] = shards[r]; sub++; }

    uint8_t* sub_m = (uint8_t*)malloc((size_t)k * k);
    uint8_t* dec = (uint8_t*)malloc((size_t)k * k);
    uint8_t* rows = (uint8_t*)malloc((size_t)m * k);
    if (!sub_m || !dec || !rows) { free(sub_m); free(dec); free(rows); return RSO_ERR_ALLOC; }
    for (int r = 0; r < k; r++) memcpy(sub_m + r * k, mat + (size_t)valid[r] * k, k);
    rc = rso_invert(k, sub_m, dec);
    if (rc) { free(sub_m); free(dec); free(rows); return rc; }

    uint8_t* outs[256];
    int cnt = 0;
    for (int i = 0; i < k; i++)
        if (!lens[i]) {
            if (!shards[i]) { free(sub_m); free(dec); free(rows); return RSO_ERR_ALLOC; }
            memcpy(rows + cnt * k, dec + i * k, k);
            outs[cnt++] = shards[i];
            lens[i] = size;
        }
    if (cnt) rso_code(rows, k, cnt, sub_shards, outs, size, 0, 1);
    if (!data_only) {
        cnt = 0;
        for (int i = k; i < n; i++)
            if (!lens[i]) {
                if (!shards[i]) { free(sub_m); free(dec); free(rows); return RSO_ERR_ALLOC; }
                memcpy(rows + cnt * k, mat + (size_t)i * k, k);
                outs[cnt++] = shards[i];
                lens[i] = size;
            }
        if (cnt) rso_code(rows, k, cnt, (const uint8_t* const*)shards, outs, size, 0, 1);
    }
    free(sub_m); free(dec); free(rows);
    return RSO_OK;
}

/* ---- CRC-32C (Castagnoli), as Go's hash/crc32 with crc32.MakeTable(crc32.Castagnoli) ----
 * Used on blb's RS data path by pkg/disk/checksum_block.go:34,70-80 (64 KiB ChecksumFile
 * blocks: 65532 data bytes + 4-byte CRC) and pkg/rpc/bulk_codec.go:47 (bulk RPC frames).
 * rso_crc32c_update = crc32.Update(crc, tab, p); Checksum(p) = Update(0, tab, p). */
static uint32_t crc32c_table[256];
static int crc32c_ready = 0;

static void crc32c_init(void) {
    if (crc32c_ready) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc32c_table[i] = c;
    }
    crc32c_ready = 1;
}

uint32_t rso_crc32c_update(uint32_t crc, const uint8_t* p, size_t n) {
    crc32c_init();
    crc = ~crc;
    for (size_t i = 0; i < n; i++) crc = crc32c_table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}

/* CRC of each `block`-byte block of p[0:n] (last block may be short). */
void rso_crc32c_blocks(const uint8_t* p, size_t n, size_t block, uint32_t* out) {
    size_t j = 0;
    for (size_t off = 0; off < n; off += block, j++)
        out[j] = rso_crc32c_update(0, p + off, (n - off < block) ? n - off : block);
}

/* ---- CRC-32C the way Go's hash/crc32 computes it on amd64 (CPU baseline only) ----
 * blb's crc32.Checksum(b, castagnoliTable) (pkg/disk/checksum_block.go:70-80) dispatches,
 * on amd64 with SSE4.2, to the standard library's castagnoliSSE42 / castagnoliSSE42Triple:
 * the crc32 instruction over three interleaved streams of a fixed stride, joined with
 * precomputed shift tables, then single-stream for the remainder.  This restates that
 * algorithm class (stride 8 KiB, one 4 x 256 shift table) so bench.py's cpu_baseline times
 * what the reference's own CPU path does; results equal rso_crc32c_blocks (the checker). */
#define CRC_TRIPLE 8192u
typedef struct { uint32_t t[4][256]; } crc_shift_tab;

__attribute__((target("sse4.2"))) static uint32_t crc_hw_stream(uint32_t c, const uint8_t* p, size_t n) {
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c = (uint32_t)_mm_crc32_u64(c, v);
        p += 8;
        n -= 8;
    }
    while (n--) c = _mm_crc32_u8(c, *p++);
    return c;
}

/* t[k][b] = register after CRC_TRIPLE zero bytes starting from b << 8k (linear in the start). */
__attribute__((target("sse4.2"))) static void crc_build_shift(crc_shift_tab* s) {
    static const uint8_t zeros[CRC_TRIPLE];
    for (int k = 0; k < 4; k++)
        for (uint32_t b = 0; b < 256; b++) s->t[k][b] = crc_hw_stream(b << (8 * k), zeros, CRC_TRIPLE);
}

static inline uint32_t crc_shift(const crc_shift_tab* s, uint32_t c) {
    return s->t[0][c & 255] ^ s->t[1][(c >> 8) & 255] ^ s->t[2][(c >> 16) & 255] ^ s->t[3][c >> 24];
}

__attribute__((target("sse4.2"))) static uint32_t crc_hw(const crc_shift_tab* s, const uint8_t* p, size_t n) {
    uint32_t c = ~0u;
    for (; n >= 3 * CRC_TRIPLE; p += 3 * CRC_TRIPLE, n -= 3 * CRC_TRIPLE) {
        uint32_t a = c, b = 0, d = 0;
        for (size_t i = 0; i < CRC_TRIPLE; i += 8) {
            uint64_t va, vb, vd;
            memcpy(&va, p + i, 8);
            memcpy(&vb, p + CRC_TRIPLE + i, 8);
            memcpy(&vd, p + 2 * CRC_TRIPLE + i, 8);
            a = (uint32_t)_mm_crc32_u64(a, va);
            b = (uint32_t)_mm_crc32_u64(b, vb);
            d = (uint32_t)_mm_crc32_u64(d, vd);
        }
        c = crc_shift(s, crc_shift(s, a) ^ b) ^ d;
    }
    return ~crc_hw_stream(c, p, n);
}

int rso_have_sse42(void) { return __builtin_cpu_supports("sse4.2"); }

/* Same output as rso_crc32c_blocks; `threads` OpenMP threads split the blocks. */
void rso_crc32c_blocks_hw(const uint8_t* p, size_t n, size_t block, uint32_t* out, int threads) {
    static crc_shift_tab s;
    static int ready = 0;
    if (!ready) {
        crc_build_shift(&s);
        ready = 1;
    }
    const long nb = (long)((n + block - 1) / block);
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
    for (long j = 0; j < nb; j++) {
        const size_t off = (size_t)j * block;
        out[j] = crc_hw(&s, p + off, (n - off < block) ? n - off : block);
    }
}
