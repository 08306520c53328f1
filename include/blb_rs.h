/*
 * blb_rs.h -- C ABI of the MI355X Reed-Solomon engine (libblbrs.so).
 *
 * Drop-in boundary for blb's use of github.com/klauspost/reedsolomon
 * (@925cb01d6510, /root/reference/go.mod:20).  blb binds exactly four methods of the Go
 * interface reedsolomon.Encoder plus the constructor:
 *
 *   reedsolomon.New(n, m)        internal/tractserver/store.go:1022, client/blb/reconstruct.go:166
 *   Encoder.Encode(shards)       internal/tractserver/store.go:1099
 *   Encoder.Reconstruct(shards)  internal/tractserver/store.go:1133
 *   Encoder.Verify(shards)       internal/tractserver/store.go:1136
 *   Encoder.ReconstructData(s)   client/blb/reconstruct.go:173
 *
 * Each of those has a host-memory entry point below with the same argument meaning and
 * error behaviour; a cgo shim marshals Go's [][]byte into the
 * (pointer, length) arrays.  The *_dev entry points are the device-resident batched path
 * used when stripes already live in HBM (bench.py, batched callers).
 *
 * Conventions (klauspost semantics, reproduced exactly):
 *   - shards[] / lens[] always have k+m entries, data shards first.
 *   - A shard with lens[i] == 0 is "missing" (Reconstruct*) -- its pointer must then be a
 *     caller buffer with room for the shard size (klauspost reslices shards[i][0:size] when
 *     cap >= size; client/blb/reconstruct.go:172-175 relies on the output landing in the
 *     caller's buffer), or NULL for a parity slot that ReconstructData will not produce.
 *   - Outputs are fully overwritten, never accumulated into (rpc.GetBuffer returns
 *     un-zeroed pooled buffers, pkg/rpc/pool.go:28-43).
 *   - No pointer is retained after a call returns (cgo rule).  A small host call may return
 *     on its kernel's completion word, before the dispatch has retired: the word is published
 *     after every output is written, and the kernel touches no caller memory after it.
 *   - All functions are thread-safe and none changes the calling thread's current HIP
 *     device.  Host-memory calls run on the least-loaded device of the encoder's device
 *     list (blbrs_new_on; blbrs_new takes the process default list), each on a stream worker
 *     of that device -- at most blbrs_set_worker_limit() workers per device, further callers
 *     wait for one.  Device-resident (*_dev) calls run on the device that owns the stripes.
 *     cgo callers therefore need no per-thread device state (goroutines migrate between OS
 *     threads).
 */
#ifndef BLB_RS_H
#define BLB_RS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes: 1:1 with klauspost's exported errors (reedsolomon.go), plus engine errors. */
#define BLBRS_OK                 0
#define BLBRS_ERR_INV_SHARD_NUM (-1) /* ErrInvShardNum: "cannot create Encoder with zero or less data/parity shards" */
#define BLBRS_ERR_MAX_SHARD_NUM (-2) /* ErrMaxShardNum: "cannot create Encoder with more than 256 data+parity shards" */
#define BLBRS_ERR_TOO_FEW_SHARDS (-3) /* ErrTooFewShards: "too few shards given" */
#define BLBRS_ERR_SHARD_NO_DATA (-4) /* ErrShardNoData: "no shard data" */
#define BLBRS_ERR_SHARD_SIZE    (-5) /* ErrShardSize: "shard sizes do not match" */
#define BLBRS_ERR_SINGULAR      (-6) /* errSingular (matrix.go): "matrix is singular" */
#define BLBRS_ERR_INVALID_ARG   (-7) /* NULL pointer / bad stride / missing output buffer */
#define BLBRS_ERR_HIP           (-8) /* HIP runtime failure; see blbrs_last_error() */
#define BLBRS_ERR_NO_DEVICE     (-9) /* no gfx950 device visible */
#define BLBRS_ERR_LIMIT        (-10) /* pinned-memory live limit reached (blbrs_pool_set_live_limit):
                                        the caller falls back to pageable memory */

typedef struct blbrs_encoder blbrs_encoder;
typedef struct blbrs_batcher blbrs_batcher;

/* Per-device runtime counters (blbrs_get_device_stats). */
typedef struct {
    uint64_t workers;        /* stream workers alive on the device (<= the worker limit) */
    uint64_t idle;           /* of which idle */
    uint64_t waits;          /* calls that had to wait for a free worker */
    uint64_t staging_bytes;  /* pinned staging memory held by the device's workers */
    uint64_t calls;          /* host-memory calls and host-batch parts run on the device */
    int64_t inflight;        /* of which running now */
    uint64_t done_waits;     /* small calls that ended on their kernel's completion word */
    uint64_t done_fallbacks; /* small calls whose word did not come within the spin bound:
                                they waited for the stream instead (which reports a fault) */
} blbrs_device_stats;

/* Pinned buffer pool counters (blbrs_get_pool_stats). */
typedef struct {
    uint64_t gets, puts;     /* blbrs_buffer_get / blbrs_buffer_put calls */
    uint64_t allocs, frees;  /* pinned allocations made / released */
    uint64_t live_bytes;     /* capacity handed out and not yet put back */
    uint64_t idle_bytes;     /* capacity kept for reuse */
    uint64_t registered_bytes; /* caller memory pinned by blbrs_buffer_register, not yet unregistered */
    uint64_t registrations;  /* blbrs_buffer_register calls that pinned memory */
    uint64_t live_limit;     /* cap on live_bytes + registered_bytes (blbrs_pool_set_live_limit) */
    uint64_t limit_rejects;  /* gets / registrations refused with BLBRS_ERR_LIMIT */
} blbrs_pool_stats;

/* Load of one lane (blbrs_encoder_lane_stats): entry i of an encoder's device list.  A
 * repeated device id is a further lane on that device ([0, 0] = two lanes on GPU 0). */
typedef struct {
    uint64_t calls;          /* host calls routed to the lane so far */
    uint64_t bytes;          /* their shard bytes (k+m shards x length) */
    int64_t inflight_calls;  /* of which running now */
    int64_t inflight_bytes;
} blbrs_lane_stats;

/* One device's share of a device-resident batch (blbrs_*_parts). */
typedef struct {
    uint8_t* stripes;        /* device memory: shard i of stripe b at stripes + b*stripe_stride + i*shard_stride */
    size_t shard_stride;
    size_t stripe_stride;
    size_t batch;            /* stripes in this part */
    void* stream;            /* a stream of the device owning `stripes`; NULL = its null stream */
} blbrs_dev_part;

/* ---- construction (reedsolomon.New) ---- */

/* reedsolomon.New(dataShards, parityShards): builds the (k+m) x k systematic matrix
 * M = V * inv(V[0:k]), V[r][c] = r^c over GF(2^8)/0x11D.  Errors: INV_SHARD_NUM when
 * k <= 0 or m <= 0, MAX_SHARD_NUM when k + m > 256. */
int blbrs_new(int data_shards, int parity_shards, blbrs_encoder** out);
/* reedsolomon.New on an explicit device list.  Host-memory calls of the encoder run on the
 * entry with the fewest shard bytes in flight; blbrs_encode_host_batch splits its stripes over
 * the entries.  Entries
 * may repeat ([0, 0] = two lanes on GPU 0).  blbrs_new(k, m) uses the process default list:
 * blbrs_set_default_devices(), else $BLBRS_DEVICES ("0,2,..."), else every visible device.
 * Device ids are checked at the first call that needs a device (INVALID_ARG / NO_DEVICE). */
int blbrs_new_on(int data_shards, int parity_shards, const int* devices, int ndevices, blbrs_encoder** out);
/* The encoder's device list (the default list resolved): *n = its length, up to cap ids
 * copied to out. */
int blbrs_encoder_devices(blbrs_encoder* enc, int* out, int cap, int* n);
/* Load of entry `lane` of the encoder's device list (shared with every encoder whose list
 * maps to the same (device, repeat) lane). */
int blbrs_encoder_lane_stats(blbrs_encoder* enc, int lane, blbrs_lane_stats* out);
/* Process default device list for blbrs_new encoders; (NULL, 0) = back to $BLBRS_DEVICES /
 * every visible device.  Encoders created earlier keep the list they resolved. */
int blbrs_set_default_devices(const int* devices, int ndevices);
void blbrs_free(blbrs_encoder* enc);
int blbrs_data_shards(const blbrs_encoder* enc);
int blbrs_parity_shards(const blbrs_encoder* enc);
/* Copies the (k+m)*k encoding matrix (row-major) into out; cap must be >= (k+m)*k. */
int blbrs_matrix(const blbrs_encoder* enc, uint8_t* out, size_t cap);
/* Which kernels run this encoder's Encode as a bit-plane XOR network instead of the v_perm
 * table multiply, one bit per kernel (each kernel has its own measured threshold):
 *   BLBRS_NET_CODE  rs_code_kernel (Encode / Verify): the parity rows compiled into the library
 *                   (gf_bitslice.hpp: k in {3,4,6,8,10,12}, m <= 5) where k + m > 9;
 *   BLBRS_NET_TILE  the fused encode+CRC tile kernel (k + m > 11);
 *   BLBRS_NET_PACK  PackTracts + Encode (k + m > 9);
 *   BLBRS_NET_RTC   rs_code_kernel with a network generated and compiled at run time (rtc.hpp:
 *                   k outside the compiled list, k + m > BLBRS_RTC_WIDE).
 * 0 = tables everywhere (also with the knob BLBRS_BITSLICE = 0).  Same bytes either way; a
 * diagnostic for tests and profiles. */
#define BLBRS_NET_CODE 1
#define BLBRS_NET_TILE 2
#define BLBRS_NET_PACK 4
#define BLBRS_NET_RTC  8
int blbrs_encoder_compiled_network(const blbrs_encoder* enc);

/* ---- host-memory Encoder methods (what the cgo shim binds) ---- */

/* Encoder.Encode: shards[0..k) in, shards[k..k+m) out.  All k+m lens equal and non-zero
 * (else SHARD_NO_DATA / SHARD_SIZE). */
int blbrs_encode(blbrs_encoder* enc, uint8_t* const* shards, const size_t* lens);

/* Encoder.Verify: *ok = 1 when the parity shards equal P * data, 0 otherwise
 * (klauspost returns (false, nil) on mismatch). */
int blbrs_verify(blbrs_encoder* enc, const uint8_t* const* shards, const size_t* lens, int* ok);

/* Encoder.Reconstruct: rebuild every missing shard (data and parity).  lens[i] is set to
 * the shard size for every slot produced.  All present: no work, OK.  Fewer than k
 * present: TOO_FEW_SHARDS.  Decode uses the first k present indices ascending. */
int blbrs_reconstruct(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens);

/* Encoder.ReconstructData: rebuild missing data shards only; parity slots untouched. */
int blbrs_reconstruct_data(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens);

/* reconstructAndVerify (internal/tractserver/store.go:1132-1142) in one device round trip
 * and one kernel pass: the missing shards are written and the present shards the decode does
 * not read are checked against it, which is what Verify after Reconstruct checks.  Same
 * arguments and errors as blbrs_reconstruct; *ok = 0 is store.go's errVerifyFailed. */
int blbrs_reconstruct_verify(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens, int* ok);

/* ---- device-resident batched path (stripes already in HBM) ----
 * Strided layout: shard i of stripe b lives at
 *     stripes + b * stripe_stride + i * shard_stride          (i in [0, k+m))
 * The *_ptrs forms take a HOST array of batch*(k+m) DEVICE pointers, stripe-major.
 * stream is a hipStream_t (NULL = default stream); calls are asynchronous on it.
 * Device: the calling thread's current HIP device. */

/* Batched Encode: parity shards k..k+m-1 of every stripe are (over)written. */
int blbrs_encode_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                     size_t stripe_stride, size_t batch, size_t shard_len, void* stream);
int blbrs_encode_dev_ptrs(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch,
                          size_t shard_len, void* stream);

/* Batched Reconstruct / ReconstructData with ONE erasure pattern for the whole batch
 * (present[i] != 0 means shard i is intact in every stripe).  Missing data shards (and,
 * unless data_only, missing parity shards) are written in place.  All rows are produced
 * in a single pass over the k surviving shards (missing parity uses P * inv(M[valid])). */
int blbrs_reconstruct_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                          size_t stripe_stride, size_t batch, size_t shard_len,
                          const uint8_t* present, int data_only, void* stream);
int blbrs_reconstruct_dev_ptrs(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch,
                               size_t shard_len, const uint8_t* present, int data_only,
                               void* stream);

/* Batched Verify: mismatch_dev is a DEVICE int32 array of batch entries; entry b is set
 * to 1 when stripe b's parity differs from P * data (entries are zeroed first). */
int blbrs_verify_dev(blbrs_encoder* enc, const uint8_t* stripes, size_t shard_stride,
                     size_t stripe_stride, size_t batch, size_t shard_len,
                     int32_t* mismatch_dev, void* stream);
int blbrs_verify_dev_ptrs(blbrs_encoder* enc, const uint8_t* const* shard_ptrs, size_t batch,
                          size_t shard_len, int32_t* mismatch_dev, void* stream);

/* Batched reconstructAndVerify (internal/tractserver/store.go:1132-1142: Reconstruct, then
 * Verify) in ONE pass over HBM, one erasure pattern for the batch: every missing shard (data
 * and parity) is written, and mismatch_dev[b] (device, zeroed first) is set to 1 when stripe
 * b fails the Verify that would follow.  The pass reads the k shards the decode uses and the
 * other present shards, and writes the missing ones: k + m shards per stripe instead of the
 * 2k + m + e of Reconstruct then Verify.  Nothing missing: a plain Verify.  The host-memory
 * blbrs_reconstruct_verify and the batcher use the same pass. */
int blbrs_reconstruct_verify_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                                 size_t stripe_stride, size_t batch, size_t shard_len,
                                 const uint8_t* present, int32_t* mismatch_dev, void* stream);

/* Multi-device batches: parts[p] is one device's share (the device that owns
 * parts[p].stripes), launched asynchronously on parts[p].stream -- the caller synchronizes
 * each part's stream.  One erasure pattern for the whole batch, as in the single-device
 * calls.  mismatch_dev[p] is a DEVICE int32 array of parts[p].batch entries on that part's
 * device. */
int blbrs_encode_parts(blbrs_encoder* enc, const blbrs_dev_part* parts, size_t nparts, size_t shard_len);
int blbrs_reconstruct_parts(blbrs_encoder* enc, const blbrs_dev_part* parts, size_t nparts, size_t shard_len,
                            const uint8_t* present, int data_only);
int blbrs_verify_parts(blbrs_encoder* enc, const blbrs_dev_part* parts, size_t nparts, size_t shard_len,
                       int32_t* const* mismatch_dev);

/* ---- streaming host path (host stripes -> GPU -> host parity) ----
 * Encodes `batch` stripes whose k+m shards are HOST pointers (shard_ptrs stripe-major).  The
 * stripes are split contiguously over the encoder's device list, one host thread per entry.
 * nstreams = 0 (the default of the language bindings): pinned (blbrs_buffer_get /
 * blbrs_host_alloc / blbrs_host_register) stripes are coded in place, the kernels reading the
 * data and writing the parity over PCIe (zero copy).  Pageable stripes are staged by CPU copies
 * through the worker's pinned, device-mapped buffer, in column chunks, so the CPU copies of one
 * chunk overlap the kernels of the next; no pageable memory is handed to a HIP copy.
 * nstreams >= 1 (at most 8 used): when every shard of a device's part is pinned, that part runs
 * the copy-engine pipeline instead: hipMemcpyAsync of each stripe's k data shards into a device
 * ring slot, the kernel on the slot, hipMemcpyAsync of its m parity shards back, stripe b on
 * stream b % nstreams.  Parts with pageable shards take the staged path above.
 * INVALID_ARG for nstreams < 0. */
int blbrs_encode_host_batch(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch,
                            size_t shard_len, int nstreams);

/* ---- pinned host memory: rpc.GetBuffer / PutBuffer (pkg/rpc/pool.go:16-62) ----
 * blb's shards come from rpc.GetBuffer: pooled, NOT zeroed, capacity classes of 1, 4 and
 * 8 MiB + disk.ExtraRoom (64 KiB).  Pinned shards are coded zero-copy (the kernels read and
 * write them over PCIe, no staging).  Two ways to get them:
 *
 * 1. Library-owned buffers (C / C++ callers with explicit or refcounted lifetime):
 *    blbrs_buffer_get returns a buffer of blb's class in pinned memory mapped for every
 *    device; *cap is the class capacity (>= n).  Besides blb's classes there is a 128 KiB +
 *    ExtraRoom class, used by the library's own staging (blb does not pool that size, and
 *    the Go shim returns make() for it).  Requests above the 8 MiB class get an exact
 *    allocation that blbrs_buffer_put frees.  Never blocks (like sync.Pool); idle buffers
 *    above the idle limit (default 4 GiB) are freed on put.  put of a pointer not from get is
 *    INVALID_ARG.  A buffer that is never put stays allocated: callers whose buffers may be
 *    dropped without a put (Go's rpc.GetBuffer users: bulk_codec.go:212-221 on a read error,
 *    reconstruct.go:126-152 stragglers) must use (2).
 * 2. Caller-owned memory (the Go shim: Go-heap buffers whose lifetime the GC decides):
 *    blbrs_buffer_register pins [p, p+n) (portable, mapped) and blbrs_buffer_unregister
 *    unpins it; the owner unregisters before the memory is freed (Go: a finalizer on the
 *    backing array).  Nothing else is retained.
 *
 * Both count against the live limit (default 16 GiB, blbrs_pool_set_live_limit; 0 = no
 * limit): live = capacity handed out and not put back + bytes registered.  A get or register
 * that would exceed it fails with BLBRS_ERR_LIMIT and pins nothing -- the caller uses pageable
 * memory instead (make()), which the engine stages.  The library's own transient staging is
 * counted but never refused. */
int blbrs_buffer_get(size_t n, uint8_t** out, size_t* cap);
int blbrs_buffer_put(uint8_t* p);
int blbrs_buffer_register(void* p, size_t n);
int blbrs_buffer_unregister(void* p);
int blbrs_pool_set_idle_limit(size_t bytes);
int blbrs_pool_set_live_limit(size_t bytes);
int blbrs_get_pool_stats(blbrs_pool_stats* out);
/* Plain pinned allocations (hipHostMalloc, portable + mapped) and registration of existing
 * host memory (hipHostRegister, portable + mapped) for callers with their own pools. */
int blbrs_host_alloc(size_t n, void** out);
int blbrs_host_free(void* p);
int blbrs_host_register(void* p, size_t n);
int blbrs_host_unregister(void* p);

/* ---- runtime limits ---- */
/* Maximum stream workers per device (default 8, >= 1).  Each holds two streams, a verify
 * flag and at most 2 x 8 MiB of pinned, device-mapped staging (pageable shards only: the CPU
 * copies them in and out; pageable memory is never handed to HIP's copy engines). */
int blbrs_set_worker_limit(int per_device);
int blbrs_get_device_stats(int device, blbrs_device_stats* out);
/* Frees idle stream workers and idle pooled buffers. */
int blbrs_trim(void);
/* Coding plans built since the process started: host plans (matrix inversions, one per (k, m)
 * and erasure pattern) and device plans (table uploads, one per host plan and device).  Plans
 * live for the process, so a client's per-read New / ReconstructData / free of the same
 * pattern (client/blb/reconstruct.go:166-173) builds and uploads once. */
int blbrs_plan_stats(uint64_t* host_plans, uint64_t* device_plans);

/* ---- diagnostics (no blb counterpart) ----
 * Registers, once per process, an HSA system-event handler that prints a GPU memory fault's
 * virtual address and reason to stderr, with the host / device ranges the library released
 * most recently near that address (pool frees and trims, unregistrations, staging and table
 * growth).  The runtime still ends the process after a fault; this only names the address. */
int blbrs_debug_watch_faults(void);

/* ---- pointer-table check ----
 * Every shard-pointer table the library uploads carries a 16-bit tag per upload in bits 48-63
 * of each entry, and the coding kernel skips (never dereferences) a stripe holding an entry
 * without its launch's tag.  Host calls and batched calls fail with BLBRS_ERR_HIP naming the
 * stripe, slot and entry.  The asynchronous *_dev_ptrs calls record it per device: after
 * synchronizing the stream, blbrs_table_fault_take reads and clears that record (*found = 0
 * when clear). */
typedef struct {
    uint32_t stripe;        /* stripe index within the launch */
    uint32_t slot;          /* shard slot within the stripe */
    uint32_t launch_tag;    /* the tag the kernel expected */
    uint32_t entry_tag;     /* the tag the entry carried */
    uint64_t address;       /* the entry's address bits */
} blbrs_table_fault;
int blbrs_table_fault_take(int device, blbrs_table_fault* out, int* found);
/* Test hook: the next tagged table upload writes entry `slot` with a wrong tag (address
 * intact), so the check above can be exercised without a bad address. */
int blbrs_debug_corrupt_next_table(int slot);

/* ---- CRC-32C (Castagnoli) of shard blocks ----
 * blb checksums every shard it writes on this path: ChecksumFile blocks of 65532 data
 * bytes (pkg/disk/checksum_block.go:18-34,70-80) and bulk RPC frames (pkg/rpc/
 * bulk_codec.go:47, block = whole buffer).  For each of `batch` buffers (buffer b at
 * data + b * stride, `len` bytes), out[b * nblocks + j] = crc32.Checksum(block j,
 * crc32.MakeTable(crc32.Castagnoli)) with nblocks = ceil(len / block); the last block of a
 * buffer may be short.  block == 0 means one block per buffer.  Blocks start at byte 0 of
 * each buffer: for a buffer that starts inside a file block use blbrs_crc32c_dev_at. */
int blbrs_crc32c_dev(const uint8_t* data, size_t stride, size_t batch, size_t len, size_t block,
                     uint32_t* out_dev, void* stream);
/* Host-memory form: one buffer; out (host) has ceil(len / block) entries.  Pinned / device
 * memory is read in place; pageable memory is copied by the CPU into pinned staging in chunks
 * of at most 8 MiB (block boundaries kept through the phase / seed continuation below), so a
 * call's staging stays within the worker bound whatever `len` is. */
int blbrs_crc32c(const uint8_t* data, size_t len, size_t block, uint32_t* out);

/* Encode fused with the CRC-32C of the parity it writes, in one pass over HBM: what
 * Store.rsEncodeOne does with each increment (Encode, store.go:1099) followed by the
 * checksum of every parity shard it ships -- the bulk RPC frame CRC of CtlWrite
 * (pkg/rpc/bulk_codec.go:47; block = 0 = whole shard) or the receiver's ChecksumFile blocks
 * (block = 65532, pkg/disk/checksum_block.go:18-34).  Same strided layout and parity bytes
 * as blbrs_encode_dev; crc_out_dev (device) receives m * batch * nblocks entries,
 * nblocks = ceil(shard_len / block):
 *     crc_out_dev[(j * batch + b) * nblocks + i] = CRC-32C of block i of parity shard k+j
 *                                                  of stripe b.
 * Shapes without a fused kernel fall back to the coding pass plus blbrs_crc32c_dev's kernel
 * (same results).  Blocks start at byte 0 of each shard; parity windows at other file
 * offsets use blbrs_encode_crc_dev_at. */
int blbrs_encode_crc_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                         size_t stripe_stride, size_t batch, size_t shard_len, size_t block,
                         uint32_t* crc_out_dev, void* stream);

/* File-aligned continuation forms of the two calls above, for buffers that are a window of a
 * file (rsEncodeOne writes parity window i at offset 4 MiB * i of the piece, store.go:1028-
 * 1037,1115, and 4 MiB mod 65532 = 256): byte 0 of every buffer sits `phase` bytes into its
 * first block (phase = file offset mod block, < block), so
 *     nblocks = ceil((phase + len) / block)
 * and block i covers the buffer bytes [max(0, i*block - phase), min(len, (i+1)*block - phase)).
 * Entry i = crc32.Update(i == 0 ? seed : 0, castagnoliTable, those bytes) -- the ChecksumFile
 * append rule b.cksum = crc32.Update(b.cksum, ...) (pkg/disk/checksum_block.go:76-81): pass
 * the CRC the file's partial last block already has as the seed (for window w+1, the last
 * entry window w produced), and block 0's entry is that block's new checksum.  seeds_dev is a
 * DEVICE array (NULL = all 0 = plain crc32.Checksum): one per buffer for blbrs_crc32c_dev_at,
 * [j * batch + b] per parity shard for blbrs_encode_crc_dev_at.  block == 0 = one block per
 * buffer (phase ignored).  phase >= block is INVALID_ARG. */
int blbrs_crc32c_dev_at(const uint8_t* data, size_t stride, size_t batch, size_t len, size_t block,
                        size_t phase, const uint32_t* seeds_dev, uint32_t* out_dev, void* stream);
int blbrs_encode_crc_dev_at(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                            size_t stripe_stride, size_t batch, size_t shard_len, size_t block,
                            size_t phase, const uint32_t* seeds_dev, uint32_t* crc_out_dev, void* stream);
/* The recovery write path: blbrs_reconstruct_dev (one erasure pattern for the batch; the
 * rebuilt shards go to the new hosts by CtlWrite, internal/tractserver/store.go:1110-1120)
 * fused with the CRC-32C of every rebuilt shard, the same block / phase / seed rules as
 * blbrs_encode_crc_dev_at.  Output row j = the j-th rebuilt shard: missing data shards
 * ascending, then (data_only == 0) missing parity shards ascending;
 * crc_out_dev[(j * batch + b) * nblocks + i], seeds_dev[j * batch + b].  Nothing missing (or
 * data_only with only parity missing): no work, no CRC written. */
int blbrs_reconstruct_crc_dev_at(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                                 size_t stripe_stride, size_t batch, size_t shard_len,
                                 const uint8_t* present, int data_only, size_t block, size_t phase,
                                 const uint32_t* seeds_dev, uint32_t* crc_out_dev, void* stream);

/* ---- batched host calls: client reconstructs and tractserver encodes (SURVEY.md §8f rows
 * 4 and 1) ----
 * client/blb/reconstruct.go:65-195 calls ReconstructData once per degraded read (one stripe
 * of `length`-byte pieces), up to MaxInFlight (:19,35-45) at once; the tractserver calls
 * Encode once per 4 MiB increment of each RSEncode RPC (store.go:1099), up to
 * RejectCtlReqThreshold = 1000 RPCs at once (internal/tractserver/config.go:91).  A batcher
 * collects concurrent host Encode / Verify / Reconstruct / ReconstructData /
 * reconstructAndVerify calls that arrive within window_us (or until max_batch wait) and runs
 * them as one kernel launch per (encoder shape, plan, length) group -- plus the verify pass
 * and its per-stripe flags for the verifying calls -- and one stream sync.  Attach it to an
 * encoder and the plain blbrs_encode / blbrs_verify / blbrs_reconstruct /
 * blbrs_reconstruct_data / blbrs_reconstruct_verify calls on that encoder go through it: same
 * arguments, results and errors, the caller still blocks until its own stripe is done -- the
 * Go Encoder interface is unchanged.  window_us = 0 batches naturally: a free lane takes whatever is
 * queued at once and calls arriving while the lanes are busy form the next batch, so a lone
 * caller does not wait; a positive window holds a batch open up to window_us after its first
 * call.
 * Pinned / device shards are used in place; pageable ones are staged by the calling thread
 * through the pinned buffer pool.  Each device of the batcher has a queue drained by two
 * lanes (own stream each), so one batch is collected while the previous one runs.  A call
 * whose shards are device memory goes to that device's queue, any other to the shortest
 * queue.  blbrs_batcher_new uses the process default device list.  Free a batcher after
 * detaching it from every encoder. */
int blbrs_batcher_new(int max_batch, int window_us, blbrs_batcher** out);
int blbrs_batcher_new_on(int max_batch, int window_us, const int* devices, int ndevices, blbrs_batcher** out);
void blbrs_batcher_free(blbrs_batcher* b);
int blbrs_encoder_set_batcher(blbrs_encoder* enc, blbrs_batcher* b); /* b = NULL detaches */
/* Counters: calls served and kernel launches issued so far. */
int blbrs_batcher_stats(const blbrs_batcher* b, uint64_t* requests, uint64_t* launches);

/* ---- PackTracts: device assembly of packed RS data pieces ----
 * The byte work of Store.PackTracts (internal/tractserver/store.go:922-994), for `npieces`
 * pieces at once.  Piece p is dst + p * dst_stride, piece_len bytes (the PackTracts
 * `length`).  It receives every extent with .piece == p at .offset (t.write(b, src.Offset),
 * store.go:957), and ZERO in every byte no extent covers: the holes before and between
 * tracts (sparse-file reads) and the pad up to piece_len (store.go:974-980).  Extents must
 * be sorted by (piece, offset), non-overlapping and end inside piece_len, which is
 * checkTractSpec (store.go:996-1009); anything else is BLBRS_ERR_INVALID_ARG.  dst and
 * every source must be device-accessible: device memory or pinned host memory
 * (hipHostMalloc / hipHostRegister), read in place over PCIe.  Asynchronous on `stream`;
 * the extent array may be reused as soon as the call returns. */
typedef struct {
    const uint8_t* src; /* the tract bytes (CtlRead reply) */
    uint64_t offset;    /* PackTractSpec.Offset */
    uint64_t length;    /* PackTractSpec.Length */
    uint64_t piece;     /* destination piece index */
} blbrs_pack_extent;
int blbrs_pack_dev(uint8_t* dst, size_t dst_stride, size_t npieces, size_t piece_len,
                   const blbrs_pack_extent* extents, size_t nextents, void* stream);

/* PackTracts fused with Encode: the curator's encPack then encEncode
 * (internal/curator/pack_tracts.go:244-292; Store.PackTracts store.go:922-994, then
 * Encoder.Encode store.go:1099) in ONE pass over HBM.  For each of `batch` strided stripes
 * (layout as blbrs_encode_dev), data shard j of stripe b is the packed piece number
 * b * k + j of `extents` (same rules as blbrs_pack_dev, piece_len = shard_len: tracts at
 * their offsets, zero elsewhere), and parity shards k..k+m-1 are its encoding.  The data
 * bytes are written once and never read back.  Same results as blbrs_pack_dev over the data
 * shards followed by blbrs_encode_dev (which is what shapes without a fused kernel run). */
int blbrs_pack_encode_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                          size_t stripe_stride, size_t batch, size_t shard_len,
                          const blbrs_pack_extent* extents, size_t nextents, void* stream);

/* ---- misc ---- */
int blbrs_set_device(int device);      /* hipSetDevice for the calling thread (the library
                                          itself never relies on it) */
int blbrs_device_count(int* count);
/* ---- NUMA placement (8-GPU hosts: two sockets, four GPUs behind each) ----
 * A host call on pool or registered buffers prefers a GPU attached to the NUMA node holding the
 * shards (recorded once per buffer), the least-loaded such lane unless it carries more than
 * 64 MiB beyond the least-loaded lane overall; other memory is routed by load alone. */
/* The node of a device's PCIe root (sysfs), -1 when unknown. */
int blbrs_device_numa_node(int device, int* node);
/* Override it (containers without sysfs; tests). */
int blbrs_set_device_numa_node(int device, int node);
/* The node recorded for the pool or registered buffer containing p, else -1. */
int blbrs_host_numa_node(const void* p, int* node);
/* The routing policy over explicit lane nodes and bytes in flight, scanning from `start`: the
 * lane index it picks for host shards on `node` (-1: none).  For tests and tools. */
int blbrs_lane_policy(const int* nodes, const int64_t* loads, size_t n, size_t start, int node, size_t* lane);

/* ---- A/B knobs and run-time networks ---- */

/* The library's tuning knobs (BLBRS_BITSLICE, BLBRS_EC_PERSISTENT, BLBRS_RTC,
 * BLBRS_RTC_WIDE, BLBRS_DONE_WORD; blb_amd/csrc/tuning.hpp), each a choice between shipped policies,
 * start from the environment, read once, and change only here -- never by setenv while the
 * library runs.  INVALID_ARG for an unknown name. */
int blbrs_set_tuning(const char* name, long value);
int blbrs_get_tuning(const char* name, long* value);

/* Decode networks generated per erasure pattern and compiled with hipRTC.
 * The library does not link hipRTC; it opens it (dlopen) when a network is first requested.
 * With BLBRS_RTC = 1 (the default since round 6) a wide decode pass of at least 2 rows
 * (k + rows > BLBRS_RTC_WIDE = 13: blb's RS(12,5) recovery RPC and multi-row ReconstructData)
 * requests its network on first use; it compiles in the background (a host-only thread, no HIP
 * call) and the pass runs the table kernel until the network is compiled; the next launch of the
 * pass then loads the code object in its own thread.  With BLBRS_RTC = 2 the first call compiles
 * and loads it; BLBRS_RTC = 0 keeps every pass on tables and hipRTC out of the process.  hipRTC
 * missing = a compile failure: tables. */
typedef struct {
    uint64_t requested;  /* networks requested (one per pass, mode, addressing, device) */
    uint64_t compiled;   /* distinct sources compiled */
    uint64_t loaded;     /* kernels loaded on a device */
    uint64_t failed;     /* compile or load failures (those passes stay on tables) */
    uint64_t pending;    /* queued, not yet compiled */
    double compile_ms;   /* total compile time */
} blbrs_rtc_stats;
int blbrs_rtc_get_stats(blbrs_rtc_stats* out);
/* Compiles (without loading; no device needed) the network kernel of rows x k coefficients in
 * mode 0 store / 1 verify / 2 store+verify, strided or pointer-table addressing: BLBRS_OK, or
 * BLBRS_ERR_HIP with the compiler log in blbrs_last_error().  The code object (an AMDGPU ELF)
 * is copied to `code` when non-NULL (cap bytes); *len gets its size.  For tests and tools. */
int blbrs_rtc_compile(int k, int rows, const uint8_t* coef, int mode, int strided, void* code, size_t cap,
                      size_t* len);
/* Waits until no network is queued or compiling (timeout_ms < 0: no limit).  BLBRS_OK when idle,
 * BLBRS_ERR_LIMIT on timeout. */
int blbrs_rtc_wait(long timeout_ms);
/* The generated network (device source) for rows x k coefficients, NUL-terminated into out
 * (cap bytes); *ops = its VALU ops per 8-dword group.  INVALID_ARG when cap is too small. */
int blbrs_rtc_network_source(int k, int rows, const uint8_t* coef, char* out, size_t cap, int* ops);

const char* blbrs_last_error(void);    /* thread-local message for the last failure */
const char* blbrs_version(void);
const char* blbrs_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* BLB_RS_H */
