//go:build drandgpu

package gpu

/*
#include "drand_gpu.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// Beacon is the part of drand's beacon.Beacon (beacon/chain.go:16-28) the checks read.
type Beacon struct {
	PreviousRound uint64
	PreviousSig   []byte // 96 B, or the 32 B genesis seed for round 1
	Round         uint64
	Signature     []byte // 96 B
}

// beaconArrays flattens a batch for the C-ABI.  A signature that is not 96 B becomes 96 zero bytes, which
// does not decode (no compression flag), so that beacon gets the reference's decode error while the rest of
// the batch is still checked (bad[i] marks it; kyber's VerifyRecovered fails on such a signature too).
func beaconArrays(bs []*Beacon) (pr, rr []uint64, ps []byte, off []uint32, sigs []byte, bad []bool) {
	n := len(bs)
	pr, rr = make([]uint64, n), make([]uint64, n)
	off = make([]uint32, n+1)
	sigs = make([]byte, 96*n)
	bad = make([]bool, n)
	for i, b := range bs {
		pr[i], rr[i] = b.PreviousRound, b.Round
		ps = append(ps, b.PreviousSig...)
		off[i+1] = uint32(len(ps))
		if len(b.Signature) == 96 {
			copy(sigs[96*i:], b.Signature)
		} else {
			bad[i] = true
		}
	}
	return
}

func u64p(v []uint64) *C.uint64_t {
	if len(v) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&v[0]))
}

func u32p(v []uint32) *C.uint32_t {
	if len(v) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&v[0]))
}

// VerifyBeacons is beacon.VerifyBeacon (beacon/chain.go:65-71) over a batch: Message on the device, then the
// batch bls.Verify against the group key.  One error per beacon (nil = valid).
func VerifyBeacons(groupKey []byte, bs []*Beacon) ([]error, error) {
	n := len(bs)
	if n == 0 {
		return nil, nil
	}
	if len(groupKey) != 48 {
		return nil, errors.New("gpu: group key of the wrong length")
	}
	pr, rr, ps, off, sigs, bad := beaconArrays(bs)
	st := notRun(n)
	if rc := C.dg_verify_beacons(ptr(groupKey), C.size_t(n), u64p(pr), u64p(rr), ptr(ps), u32p(off), ptr(sigs),
		ptr(st), 0); rc != 0 {
		return nil, cErr("dg_verify_beacons", rc)
	}
	out := make([]error, n)
	for i, v := range st {
		if bad[i] {
			out[i] = fmt.Errorf("gpu: round %d: signature of %d bytes", bs[i].Round, len(bs[i].Signature))
		} else if v != C.DG_ST_OK {
			out[i] = fmt.Errorf("gpu: round %d: invalid beacon (status %d)", bs[i].Round, v)
		}
	}
	return out, nil
}

// SyncBatch is one batch of syncFrom's loop (beacon/beacon.go:557-602) for rounds streamed by one peer:
// the link check against the last stored round (:561-573) and VerifyRecovered of every round (:575).  It
// returns how many leading beacons may be stored: the reference stores every reply before the first bad
// one and stops there (:575-587), so a malformed reply (a signature that is not 96 B) ends the prefix at
// its own position instead of failing the whole batch.
func SyncBatch(groupKey []byte, curRound uint64, curSig []byte, bs []*Beacon) (int, error) {
	n := len(bs)
	if n == 0 {
		return 0, nil
	}
	pr, rr, ps, off, sigs, _ := beaconArrays(bs)
	links := notRun(n)
	if rc := C.dg_check_links(C.uint64_t(curRound), ptr(curSig), C.size_t(len(curSig)), C.size_t(n), u64p(pr), u64p(rr),
		ptr(ps), u32p(off), ptr(sigs), ptr(links)); rc != 0 {
		return 0, cErr("dg_check_links", rc)
	}
	verdicts, err := VerifyBeacons(groupKey, bs)
	if err != nil {
		return 0, err
	}
	for i := range bs {
		if links[i] != 0 || verdicts[i] != nil {
			return i, nil
		}
	}
	return n, nil
}

// Randomness is RandomnessFromSignature (beacon/chain.go:52-55) over a batch.
func Randomness(sigs [][]byte) ([][]byte, error) {
	s, err := flatten(sigs, 96)
	if err != nil || len(sigs) == 0 {
		return nil, err
	}
	out := make([]byte, 32*len(sigs))
	if rc := C.dg_randomness(C.size_t(len(sigs)), ptr(s), ptr(out)); rc != 0 {
		return nil, cErr("dg_randomness", rc)
	}
	r := make([][]byte, len(sigs))
	for i := range r {
		r[i] = out[32*i : 32*(i+1)]
	}
	return r, nil
}
