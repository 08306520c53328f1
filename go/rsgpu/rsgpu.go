// Package rsgpu is the cgo binding of libblbrs.so (include/blb_rs.h): a drop-in
// reedsolomon.Encoder for blb whose Encode / Verify / Reconstruct / ReconstructData run on
// MI355X HIP kernels.
//
// It replaces github.com/klauspost/reedsolomon (@925cb01d6510, blb go.mod:20) at blb's call
// sites without changing their call surface:
//
//	internal/tractserver/store.go:1022   enc, e := reedsolomon.New(N, M)  ->  rsgpu.New(N, M)
//	client/blb/reconstruct.go:166        enc, e := reedsolomon.New(n, m)  ->  rsgpu.New(n, m)
//
// and, so that the shards those calls see are pinned and coded in place over PCIe, blb's RPC
// buffer pool:
//
//	pkg/rpc/pool.go:30   GetBuffer(n)            ->  rsgpu.GetBuffer(n)
//	pkg/rpc/pool.go:51   PutBuffer(b, exclusive) ->  rsgpu.PutBuffer(b, exclusive)
//
// (the pool keeps pool.go's Go-heap buffers and GC lifetime; it only pins them -- see below)
//
// Every encoder spreads its calls over all visible GPUs (the library picks the least-loaded
// device per call; no goroutine or OS thread carries device state).  NewOn binds an encoder
// to an explicit device list.
//
// The returned value satisfies reedsolomon.Encoder (store.go:1042,1132 take that type).
// Split / Join / Update are not on blb's path; they are delegated to klauspost's CPU encoder,
// built on first use only.
//
// Source only in this repository: this image has no Go toolchain (SURVEY.md §0.4).  Build
// where Go >= 1.21 (runtime.Pinner) and the library exist:
//
//	CGO_CFLAGS=-I<repo>/include CGO_LDFLAGS="-L<repo>/blb_amd -lblbrs -Wl,-rpath,<repo>/blb_amd" go build
package rsgpu

/*
#cgo LDFLAGS: -lblbrs
#include <stdlib.h>
#include <stdint.h>
#include "blb_rs.h"
*/
import "C"

import (
	"errors"
	"io"
	"runtime"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/klauspost/reedsolomon"
)

// batcher, when set by EnableBatching, is attached to every encoder New returns.
var batcher atomic.Pointer[C.blbrs_batcher]

// errSingular carries klauspost's message for a singular decode matrix ("matrix is
// singular", matrix.go).  It is declared here because the pinned module version keeps its
// own value unexported; callers only log it (store.go:1105, reconstruct.go:177).
var errSingular = errors.New("matrix is singular")

// call runs one C entry point with the goroutine locked to its OS thread, so that the
// thread-local message blbrs_last_error() reports belongs to this call.
func call(f func() C.int) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	return mapErr(f())
}

// Map the C ABI's codes (blb_rs.h) back onto klauspost's exported error values, so
// callers comparing against reedsolomon.ErrTooFewShards etc. keep working.  Must run on
// the OS thread that made the failing call (see call).
func mapErr(rc C.int) error {
	switch rc {
	case C.BLBRS_OK:
		return nil
	case C.BLBRS_ERR_INV_SHARD_NUM:
		return reedsolomon.ErrInvShardNum
	case C.BLBRS_ERR_MAX_SHARD_NUM:
		return reedsolomon.ErrMaxShardNum
	case C.BLBRS_ERR_TOO_FEW_SHARDS:
		return reedsolomon.ErrTooFewShards
	case C.BLBRS_ERR_SHARD_NO_DATA:
		return reedsolomon.ErrShardNoData
	case C.BLBRS_ERR_SHARD_SIZE:
		return reedsolomon.ErrShardSize
	case C.BLBRS_ERR_SINGULAR:
		return errSingular
	default:
		return errors.New("rsgpu: " + C.GoString(C.blbrs_last_error()))
	}
}

// EnableBatching makes every encoder created afterwards route its Encode / Verify /
// Reconstruct / ReconstructData calls through one process-wide batcher over all visible GPUs (blb_rs.h:
// blbrs_batcher_new): concurrent degraded reads (client/blb/reconstruct.go with
// ReconstructBehavior.MaxInFlight > 1) and the increments of concurrent RSEncode RPCs
// (internal/tractserver/store.go:1099, and reconstructAndVerify's Reconstruct + Verify at
// :1132-1142) then share kernel launches.
// Call once at process start-up, before coding begins; windowMicros = 0 batches naturally
// (no added wait for a lone caller).
func EnableBatching(maxBatch, windowMicros int) error {
	var b *C.blbrs_batcher
	if err := call(func() C.int { return C.blbrs_batcher_new(C.int(maxBatch), C.int(windowMicros), &b) }); err != nil {
		return err
	}
	if !batcher.CompareAndSwap(nil, b) {
		C.blbrs_batcher_free(b)
		return errors.New("rsgpu: batching already enabled")
	}
	return nil
}

// SetWorkerLimit caps the stream workers per GPU (blbrs_set_worker_limit; default 8).
// Calls beyond the cap wait for a worker, the way the tractserver's pendingSem bounds RPCs.
func SetWorkerLimit(perDevice int) error {
	return call(func() C.int { return C.blbrs_set_worker_limit(C.int(perDevice)) })
}

// ---- pinned buffer pool: pkg/rpc/pool.go's GetBuffer / PutBuffer ----
//
// blb's pool is three sync.Pools of Go-heap buffers, and blb relies on the GC for buffers it
// never puts back: client/blb/reconstruct.go:126-152 puts back only the first n good replies
// (errored and straggling ones are dropped after cancel()), bulk_codec.go:212-221 returns on
// a read error with the buffer it took.  So this pool hands out Go memory, exactly as
// pool.go does, and pins the buffers its pools create: a new class buffer is registered with
// the engine (blbrs_buffer_register: pinned, mapped for every GPU, so Encode / Reconstruct*
// code shards on it in place) and carries a finalizer on its backing array that unregisters
// it before the GC frees it.  A dropped buffer is therefore unpinned when it is collected,
// and the pinned bytes alive at once are capped by the engine's live limit
// (SetPinnedLimit): past it registration is refused and the buffer stays pageable -- correct,
// only staged by the engine -- and is registered again when the pool hands it out later.
// Small (<= 128 KiB + ExtraRoom) and large (> the 8 MiB class) requests get make(), as in
// pool.go -- small ones come from a pinned class pool too after SetPoolSmall(true).  The engine keeps the registered address only while the buffer is alive, and only
// coding calls (during which the caller holds the slice) touch the memory.

const (
	extraRoom  = 64 << 10 // disk.ExtraRoom
	smallMax   = 128<<10 + extraRoom
	buf1MBSize = 1<<20 + extraRoom
	buf4MBSize = 4<<20 + extraRoom
	buf8MBSize = 8<<20 + extraRoom
)

var (
	// SetPoolSmall: requests of up to smallMax come from a pool too (off by default, as in
	// pool.go).
	poolSmall    atomic.Bool
	bufSmallPool = sync.Pool{New: func() interface{} { return newPinned(smallMax) }}
	buf8MBPool   = sync.Pool{New: func() interface{} { return newPinned(buf8MBSize) }}
	buf4MBPool = sync.Pool{New: func() interface{} { return newPinned(buf4MBSize) }}
	buf1MBPool = sync.Pool{New: func() interface{} { return newPinned(buf1MBSize) }}
	// The class buffers this pool allocated, by base address (a uintptr key keeps nothing
	// alive).  Only these are ever registered: a foreign slice put back with a class
	// capacity (pool.go allows any buffer) stays as it is.
	owned sync.Map // uintptr -> *poolBuf
)

type poolBuf struct{ pinned atomic.Bool }

// newPinned allocates a class buffer, ties its bookkeeping to the GC and pins it if the live
// limit allows.  The finalizer runs when the backing array is unreachable, before its memory
// is freed: it unpins the buffer (the engine keeps the registered address only until then;
// coding calls touch the memory only while their caller holds the slice).
func newPinned(size int) interface{} {
	b := make([]byte, size)
	p := &b[0]
	pb := &poolBuf{}
	owned.Store(uintptr(unsafe.Pointer(p)), pb)
	runtime.SetFinalizer(p, func(p *byte) {
		if v, ok := owned.LoadAndDelete(uintptr(unsafe.Pointer(p))); ok && v.(*poolBuf).pinned.Load() {
			C.blbrs_buffer_unregister(unsafe.Pointer(p))
		}
	})
	pin(b, pb)
	return &b
}

// pin registers a whole class buffer with the engine (BLBRS_ERR_LIMIT or no GPU: it stays
// pageable, which the engine stages).
func pin(b []byte, pb *poolBuf) {
	if C.blbrs_buffer_register(unsafe.Pointer(&b[0]), C.size_t(len(b))) == C.BLBRS_OK {
		pb.pinned.Store(true)
	}
}

func getClass(pool *sync.Pool, n int) []byte {
	b := *pool.Get().(*[]byte)
	b = b[:cap(b)] // a put slice may be shorter; its cap is the class size
	if v, ok := owned.Load(uintptr(unsafe.Pointer(&b[0]))); ok && !v.(*poolBuf).pinned.Load() {
		pin(b, v.(*poolBuf)) // refused earlier: try again now that it is reused
	}
	return b[:n]
}

// GetBuffer returns a []byte with length n and capacity >= n.  The buffer may not be zeroed!
// (pkg/rpc/pool.go:28-43.)  Buffers of the 1, 4 and 8 MiB classes are pinned while the live
// limit allows.
func GetBuffer(n int) []byte {
	if n <= smallMax {
		if n > 0 && poolSmall.Load() {
			return getClass(&bufSmallPool, n)
		}
		return make([]byte, n)
	} else if n <= buf1MBSize {
		return getClass(&buf1MBPool, n)
	} else if n <= buf4MBSize {
		return getClass(&buf4MBPool, n)
	} else if n <= buf8MBSize {
		return getClass(&buf8MBPool, n)
	}
	return make([]byte, n)
}

// PutBuffer returns a buffer to the pool (pkg/rpc/pool.go:45-62).  It is fine to call on any
// buffer that is not used again, and fine not to call at all: the GC unpins what it collects.
func PutBuffer(b []byte, exclusive bool) {
	if !exclusive {
		return
	}
	switch cap(b) {
	case smallMax:
		if poolSmall.Load() {
			bufSmallPool.Put(&b)
		}
	case buf8MBSize:
		buf8MBPool.Put(&b)
	case buf4MBSize:
		buf4MBPool.Put(&b)
	case buf1MBSize:
		buf1MBPool.Put(&b)
	}
}

// SetPoolSmall makes GetBuffer pool (and pin) requests of up to 128 KiB + ExtraRoom as well,
// which pool.go hands out as plain make() buffers.  Small replies are then coded in place
// instead of staged by CPU copies: a 64 KiB degraded read 31 -> 25 us, 128 KiB 53 -> 41 us
// with cold inputs (DESIGN.md §4d round 6; blb_amd/rpc.py set_pool_small is the same rule).
func SetPoolSmall(on bool) { poolSmall.Store(on) }

// SetPinnedLimit caps the bytes pinned at once (blbrs_pool_set_live_limit; default 16 GiB,
// 0 = no cap).  Buffers the pool creates beyond it are plain Go memory.
func SetPinnedLimit(bytes int64) error {
	return call(func() C.int { return C.blbrs_pool_set_live_limit(C.size_t(bytes)) })
}

// ChecksumBlocks returns crc32.Checksum(block, castagnoliTable) for every `block`-byte block
// of b (block 0 = the whole buffer): the 65532-byte ChecksumFile blocks of
// pkg/disk/checksum_block.go:18-34 and the bulk frame CRC of pkg/rpc/bulk_codec.go:47,
// computed on the GPU (blb_rs.h: blbrs_crc32c).
func ChecksumBlocks(b []byte, block int) ([]uint32, error) {
	if len(b) == 0 {
		return nil, nil
	}
	if block <= 0 {
		block = len(b)
	}
	out := make([]uint32, (len(b)+block-1)/block)
	var pin runtime.Pinner
	pin.Pin(&b[0])
	pin.Pin(&out[0])
	defer pin.Unpin()
	err := call(func() C.int {
		return C.blbrs_crc32c((*C.uint8_t)(unsafe.Pointer(&b[0])), C.size_t(len(b)), C.size_t(block),
			(*C.uint32_t)(unsafe.Pointer(&out[0])))
	})
	return out, err
}

type encoder struct {
	h       *C.blbrs_encoder
	k       int
	m       int
	cpuOnce sync.Once
	cpu     reedsolomon.Encoder // Split / Join / Update only, built on first use
	cpuErr  error
}

// New is reedsolomon.New(dataShards, parityShards) backed by the GPU engine, spreading its
// calls over every visible GPU ($BLBRS_DEVICES narrows the list).
func New(dataShards, parityShards int) (reedsolomon.Encoder, error) {
	var h *C.blbrs_encoder
	if err := call(func() C.int { return C.blbrs_new(C.int(dataShards), C.int(parityShards), &h) }); err != nil {
		return nil, err
	}
	return wrap(h, dataShards, parityShards), nil
}

// NewOn is New bound to an explicit device list (entries may repeat).
func NewOn(dataShards, parityShards int, devices []int) (reedsolomon.Encoder, error) {
	if len(devices) == 0 {
		return New(dataShards, parityShards)
	}
	devs := make([]C.int, len(devices))
	for i, d := range devices {
		devs[i] = C.int(d)
	}
	var h *C.blbrs_encoder
	err := call(func() C.int {
		return C.blbrs_new_on(C.int(dataShards), C.int(parityShards), &devs[0], C.int(len(devs)), &h)
	})
	if err != nil {
		return nil, err
	}
	return wrap(h, dataShards, parityShards), nil
}

func wrap(h *C.blbrs_encoder, k, m int) *encoder {
	if b := batcher.Load(); b != nil {
		C.blbrs_encoder_set_batcher(h, b)
	}
	e := &encoder{h: h, k: k, m: m}
	runtime.SetFinalizer(e, func(e *encoder) { C.blbrs_free(e.h) })
	return e
}

func (e *encoder) cpuEncoder() (reedsolomon.Encoder, error) {
	e.cpuOnce.Do(func() { e.cpu, e.cpuErr = reedsolomon.New(e.k, e.m) })
	return e.cpu, e.cpuErr
}

// marshal builds C arrays of shard pointers and lengths.  cgo forbids storing Go pointers
// in C memory unless they are pinned, so every non-empty shard is pinned with runtime.Pinner
// for the call -- pool buffers included: they are Go-heap memory (GetBuffer below), and their
// HIP registration (page-locked for DMA) is a different thing from cgo's pinning rule.  The
// C side does not retain any pointer after returning.  A missing shard that has capacity (klauspost reslices
// shards[i][0:size] when cap >= size; client/blb/reconstruct.go:172 relies on it) passes its
// backing array as the output buffer.
type marshalled struct {
	ptrs   *unsafe.Pointer
	lens   *C.size_t
	pinner runtime.Pinner
}

func marshal(shards [][]byte, size int) *marshalled {
	n := len(shards)
	mm := &marshalled{
		ptrs: (*unsafe.Pointer)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))),
		lens: (*C.size_t)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0))))),
	}
	ptrs := unsafe.Slice(mm.ptrs, n)
	lens := unsafe.Slice(mm.lens, n)
	for i, s := range shards {
		lens[i] = C.size_t(len(s))
		ptrs[i] = nil
		if cap(s) > 0 && (len(s) > 0 || cap(s) >= size) {
			p := &s[:1][0]
			mm.pinner.Pin(p)
			ptrs[i] = unsafe.Pointer(p)
		}
	}
	return mm
}

func (mm *marshalled) free() {
	mm.pinner.Unpin()
	C.free(unsafe.Pointer(mm.ptrs))
	C.free(unsafe.Pointer(mm.lens))
}

func shardSize(shards [][]byte) int {
	for _, s := range shards {
		if len(s) != 0 {
			return len(s)
		}
	}
	return 0
}

func (e *encoder) Encode(shards [][]byte) error {
	if len(shards) != e.k+e.m {
		return reedsolomon.ErrTooFewShards
	}
	mm := marshal(shards, shardSize(shards))
	defer mm.free()
	return call(func() C.int { return C.blbrs_encode(e.h, (**C.uint8_t)(unsafe.Pointer(mm.ptrs)), mm.lens) })
}

func (e *encoder) Verify(shards [][]byte) (bool, error) {
	if len(shards) != e.k+e.m {
		return false, reedsolomon.ErrTooFewShards
	}
	mm := marshal(shards, shardSize(shards))
	defer mm.free()
	var ok C.int
	err := call(func() C.int {
		return C.blbrs_verify(e.h, (**C.uint8_t)(unsafe.Pointer(mm.ptrs)), mm.lens, &ok)
	})
	if err != nil {
		return false, err
	}
	return ok != 0, nil
}

func (e *encoder) reconstruct(shards [][]byte, dataOnly bool) error {
	if len(shards) != e.k+e.m {
		return reedsolomon.ErrTooFewShards
	}
	size := shardSize(shards)
	present := 0
	for _, s := range shards {
		if len(s) != 0 {
			present++
		}
	}
	// klauspost allocates a missing output whose cap is too small -- only once the
	// argument checks have passed; do the same so the C side always has a buffer (data
	// slots always, parity slots unless dataOnly).  Error cases fall through to C.
	if size > 0 && present >= e.k && present < e.k+e.m {
		for i := range shards {
			if len(shards[i]) == 0 && cap(shards[i]) < size && (i < e.k || !dataOnly) {
				shards[i] = make([]byte, 0, size)
			}
		}
	}
	mm := marshal(shards, size)
	defer mm.free()
	err := call(func() C.int {
		if dataOnly {
			return C.blbrs_reconstruct_data(e.h, (**C.uint8_t)(unsafe.Pointer(mm.ptrs)), mm.lens)
		}
		return C.blbrs_reconstruct(e.h, (**C.uint8_t)(unsafe.Pointer(mm.ptrs)), mm.lens)
	})
	if err != nil {
		return err
	}
	lens := unsafe.Slice(mm.lens, len(shards))
	for i := range shards {
		if len(shards[i]) == 0 && lens[i] != 0 {
			shards[i] = shards[i][0:size] // output landed in the caller's backing array
		}
	}
	return nil
}

func (e *encoder) Reconstruct(shards [][]byte) error     { return e.reconstruct(shards, false) }
func (e *encoder) ReconstructData(shards [][]byte) error { return e.reconstruct(shards, true) }

func (e *encoder) Update(shards [][]byte, newDatashards [][]byte) error {
	cpu, err := e.cpuEncoder()
	if err != nil {
		return err
	}
	return cpu.Update(shards, newDatashards)
}

func (e *encoder) Split(data []byte) ([][]byte, error) {
	cpu, err := e.cpuEncoder()
	if err != nil {
		return nil, err
	}
	return cpu.Split(data)
}

func (e *encoder) Join(dst io.Writer, shards [][]byte, outSize int) error {
	cpu, err := e.cpuEncoder()
	if err != nil {
		return err
	}
	return cpu.Join(dst, shards, outSize)
}
