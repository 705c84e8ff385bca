//go:build drandgpu

// Package gpu is the drop-in of libdrandgpu.so (include/drand_gpu.h) behind drand's signature scheme:
// it implements kyber's sign.ThresholdScheme, the interface key.Scheme has (key/curve.go:30) and
// beacon.Config.Scheme receives (beacon/beacon.go:33; core/drand.go:335), plus batch methods with no
// reference counterpart.
//
// Fail closed: every C return code is checked and turned into a Go error, and every status buffer starts
// at a non-OK value, so a failed call can never read as an accepted signature.  Single-item calls stay on
// the CPU kyber scheme (latency: a GPU batch is milliseconds); batches of at least MinBatch items go to the
// GPU.
//
// EXPERIMENTAL, behind the `drandgpu` build tag: Go is not installed in the image this was written in, so
// the package has never been compiled by cgo nor checked against sign.ThresholdScheme at the kyber version
// go.mod pins; only its C calls are compile-checked, against the header, by tests/native/abi_caller.cpp.
// Build it with `go build -tags drandgpu` once it has been compiled and tested against the reference.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#cgo LDFLAGS: -L${SRCDIR}/../drand_amd -ldrandgpu -Wl,-rpath,${SRCDIR}/../drand_amd
#include "drand_gpu.h"
#include <stdlib.h>
*/
import "C"

import (
	"bytes"
	"errors"
	"fmt"
	"sync"
	"unsafe"

	"github.com/drand/kyber"
	"github.com/drand/kyber/share"
	"github.com/drand/kyber/sign"
	"github.com/drand/kyber/sign/tbls"
)

// MinBatch is the smallest batch sent to the GPU; smaller ones use the CPU scheme.
var MinBatch = 64

// stNotRun pre-fills status buffers: neither DG_ST_OK nor any code the library writes.
const stNotRun = 0xFE

var (
	initOnce sync.Once
	initErr  error
)

// Init selects the HIP device of this process (one process per GPU).
func Init(device int) error {
	initOnce.Do(func() {
		if rc := C.dg_init(C.int(device)); rc != 0 {
			initErr = cErr("dg_init", rc)
		}
	})
	return initErr
}

func cErr(fn string, rc C.int) error {
	return fmt.Errorf("gpu: %s failed (%d): %s", fn, int(rc), C.GoString(C.dg_last_error()))
}

// SetHashDST switches the hash-to-G2 domain-separation tag of every sign / verify / recover call
// (dg_set_hash_dst).  drand's suite (github.com/drand/bls12-381 v0.2.0, key/curve.go:12) predates RFC 9380;
// its DST is not pinned by any file of the reference, so a maintainer sets it here without a rebuild.
func SetHashDST(dst []byte) error {
	if rc := C.dg_set_hash_dst(ptr(dst), C.size_t(len(dst))); rc != 0 {
		return cErr("dg_set_hash_dst", rc)
	}
	return nil
}

// Scheme implements sign.ThresholdScheme over libdrandgpu (the key/curve.go:30 replacement).
type Scheme struct {
	cpu sign.ThresholdScheme // kyber's scheme: Sign (secret material) and every single-item call
}

// New wraps the CPU scheme; Init must have succeeded.
func New(cpu sign.ThresholdScheme) *Scheme { return &Scheme{cpu: cpu} }

func bytesOf(p kyber.Point) ([]byte, error) { return p.MarshalBinary() }

func commits(pub *share.PubPoly) ([]byte, error) {
	_, cs := pub.Info()
	out := make([]byte, 0, 48*len(cs))
	for _, c := range cs {
		b, err := bytesOf(c)
		if err != nil {
			return nil, err
		}
		out = append(out, b...)
	}
	return out, nil
}

func ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func notRun(n int) []byte {
	st := make([]byte, n)
	for i := range st {
		st[i] = stNotRun
	}
	return st
}

// Sign: beacon/beacon.go:433 -- the CPU kyber path (secret key material, one call per round).
func (s *Scheme) Sign(private *share.PriShare, msg []byte) ([]byte, error) { return s.cpu.Sign(private, msg) }

// IndexOf: beacon/beacon.go:154, beacon/round_cache.go:113.
func (s *Scheme) IndexOf(sig []byte) (int, error) { return s.cpu.IndexOf(sig) }

// VerifyRecovered: beacon/beacon.go:494,575, beacon/chain.go:70, core/client_public.go:116 (one item: CPU).
func (s *Scheme) VerifyRecovered(public kyber.Point, msg, sig []byte) error {
	return s.cpu.VerifyRecovered(public, msg, sig)
}

// VerifyPartial: beacon/beacon.go:148 (one item: CPU).
func (s *Scheme) VerifyPartial(public *share.PubPoly, msg, sig []byte) error {
	return s.cpu.VerifyPartial(public, msg, sig)
}

// Recover: beacon/beacon.go:488 (one round: CPU).  See RecoverVerified for the live round.
func (s *Scheme) Recover(public *share.PubPoly, msg []byte, sigs [][]byte, t, n int) ([]byte, error) {
	return s.cpu.Recover(public, msg, sigs, t, n)
}

// ---- batch extensions (no reference counterpart): what the GPU exists for.

func flatten(items [][]byte, size int) ([]byte, error) {
	out := make([]byte, 0, size*len(items))
	for _, x := range items {
		if len(x) != size {
			return nil, fmt.Errorf("gpu: item of %d bytes, want %d", len(x), size)
		}
		out = append(out, x...)
	}
	return out, nil
}

// VerifyRecoveredBatch returns one error (nil = valid) per signature: kyber's bls.Verify verdict for every rejected
// signature (each failed its own exact check); an accepted one passed a random-linear-combination batch or group test,
// which a bad signature survives with probability <= 2^-63 (drand_gpu.h Conventions).
func (s *Scheme) VerifyRecoveredBatch(public kyber.Point, msgs, sigs [][]byte) ([]error, error) {
	n := len(msgs)
	if n != len(sigs) {
		return nil, errors.New("gpu: msgs and sigs differ in length")
	}
	out := make([]error, n)
	if n < MinBatch {
		for i := range msgs {
			out[i] = s.cpu.VerifyRecovered(public, msgs[i], sigs[i])
		}
		return out, nil
	}
	m, err := flatten(msgs, len(msgs[0]))
	if err != nil {
		return nil, err
	}
	g := make([]byte, 0, 96*n)
	for i := range sigs {
		if len(sigs[i]) != 96 { // kyber's decode fails on any other length
			g = append(g, make([]byte, 96)...)
			out[i] = errors.New("gpu: signature has the wrong length")
			continue
		}
		g = append(g, sigs[i]...)
	}
	pk, err := bytesOf(public)
	if err != nil {
		return nil, err
	}
	st := notRun(n)
	if rc := C.dg_verify(ptr(pk), C.size_t(n), ptr(m), C.size_t(len(msgs[0])), ptr(g), ptr(st), 0); rc != 0 {
		return nil, cErr("dg_verify", rc)
	}
	for i := range st {
		if out[i] == nil && st[i] != C.DG_ST_OK {
			out[i] = fmt.Errorf("gpu: invalid signature (status %d)", st[i])
		}
	}
	return out, nil
}

// VerifyPartialBatch: msgs[r] and partials[r][j] (98 B each, k per round) -> one error per partial.
func (s *Scheme) VerifyPartialBatch(public *share.PubPoly, msgs [][]byte, partials [][][]byte) ([][]error, error) {
	R := len(msgs)
	if R == 0 {
		return nil, nil
	}
	k := len(partials[0])
	out := make([][]error, R)
	if R*k < MinBatch {
		for r := range msgs {
			out[r] = make([]error, k)
			for j := range partials[r] {
				out[r][j] = s.cpu.VerifyPartial(public, msgs[r], partials[r][j])
			}
		}
		return out, nil
	}
	m, err := flatten(msgs, len(msgs[0]))
	if err != nil {
		return nil, err
	}
	// a partial of the wrong length is an error of its own (kyber's VerifyPartial fails to parse it), not of the
	// batch: its error comes from the CPU scheme and a never-valid placeholder record takes its slot
	p, short, err := packPartials(partials, k)
	if err != nil {
		return nil, err
	}
	c, err := commits(public)
	if err != nil {
		return nil, err
	}
	st := notRun(R * k)
	if rc := C.dg_verify_partials(ptr(c), C.uint32_t(len(c)/48), C.size_t(R), ptr(m), C.size_t(len(msgs[0])),
		C.uint32_t(k), ptr(p), ptr(st), 0); rc != 0 {
		return nil, cErr("dg_verify_partials", rc)
	}
	for r := range out {
		out[r] = make([]error, k)
		for j := 0; j < k; j++ {
			if short[r*k+j] {
				out[r][j] = s.cpu.VerifyPartial(public, msgs[r], partials[r][j])
				if out[r][j] == nil { // cannot happen for a wrong-length share; never report it valid
					out[r][j] = errors.New("gpu: partial of the wrong length")
				}
			} else if v := st[r*k+j]; v != C.DG_ST_OK {
				out[r][j] = fmt.Errorf("gpu: invalid partial signature (status %d)", v)
			}
		}
	}
	return out, nil
}

// placeholder98 stands in for a partial of the wrong length: index 0 and a sigma whose first byte lacks the
// compression flag, which the library reports as a decode error (DG_ST_SIG_DECODE) -- never valid, so Recover
// skips it as kyber's tbls.Recover skips a partial that fails VerifyPartial.
var placeholder98 = make([]byte, 98)

// packPartials lays out R rounds of k partials as 98 B records; short[i] marks a partial of the wrong length,
// replaced by placeholder98.
func packPartials(partials [][][]byte, k int) ([]byte, []bool, error) {
	p := make([]byte, 0, 98*len(partials)*k)
	short := make([]bool, len(partials)*k)
	for r := range partials {
		if len(partials[r]) != k {
			return nil, nil, errors.New("gpu: rounds with different partial counts")
		}
		for j, x := range partials[r] {
			if len(x) != 98 {
				short[r*k+j] = true
				x = placeholder98
			}
			p = append(p, x...)
		}
	}
	return p, short, nil
}

// RecoverBatch: tbls.Recover per round (first t valid partials in input order, deduplicated by index,
// Lagrange at 0).  Returns the recovered signatures and one error per round (nil = recovered).
func (s *Scheme) RecoverBatch(public *share.PubPoly, msgs [][]byte, partials [][][]byte, t, n int) ([][]byte, []error, error) {
	R := len(msgs)
	if R == 0 {
		return nil, nil, nil
	}
	k := len(partials[0])
	m, err := flatten(msgs, len(msgs[0]))
	if err != nil {
		return nil, nil, err
	}
	// a wrong-length partial is skipped, as tbls.Recover skips a partial that fails VerifyPartial
	p, _, err := packPartials(partials, k)
	if err != nil {
		return nil, nil, err
	}
	c, err := commits(public)
	if err != nil {
		return nil, nil, err
	}
	sig := make([]byte, 96*R)
	rs, ss := notRun(R), notRun(R*k)
	if rc := C.dg_recover(ptr(c), C.uint32_t(len(c)/48), C.uint32_t(n), C.size_t(R), ptr(m), C.size_t(len(msgs[0])),
		C.uint32_t(k), ptr(p), ptr(sig), ptr(rs), ptr(ss), 0); rc != 0 {
		return nil, nil, cErr("dg_recover", rc)
	}
	return splitRecover(sig, rs, R)
}

// Verdict is a VerifyPartial verdict ProcessBeacon already holds for a partial (beacon/beacon.go:148), with
// the message it was computed against: the message of the packet's own PreviousSig (:146).
type Verdict struct {
	Err error  // nil = valid
	Msg []byte // the message the verdict is for
}

// RecoverVerified is the live round (beacon/beacon.go:472-494): ProcessBeacon already ran VerifyPartial on
// every partial the round cache holds (beacon/beacon.go:148, round_cache.go:113-119), and kyber's Recover
// (:488) would verify each of them again, against the node's own msg.  A verdict is reused only when it was
// computed against msg: the round cache admits a partial on PreviousRound alone (round_cache.go:40-48), so a
// packet built on another PreviousSig carries a verdict for another message; such partials are verified
// here against msg (kyber, CPU: the rare case), as Recover would.  Invalid ones are skipped as Recover skips
// them.  No pairing runs on the GPU.
func (s *Scheme) RecoverVerified(public *share.PubPoly, msg []byte, partials [][]byte, verified []Verdict, t, n int) ([]byte, error) {
	k := len(partials)
	if k != len(verified) {
		return nil, errors.New("gpu: partials and verdicts differ in length")
	}
	if k == 0 {
		return nil, errors.New("gpu: not enough good public shares")
	}
	p := make([]byte, 0, 98*k)
	vst := make([]byte, k)
	for j, x := range partials {
		if len(x) != 98 {
			p = append(p, make([]byte, 98)...)
			vst[j] = C.DG_ST_SIG_DECODE
			continue
		}
		p = append(p, x...)
		err := verified[j].Err
		if !bytes.Equal(verified[j].Msg, msg) {
			err = s.cpu.VerifyPartial(public, msg, x) // a verdict for another message is no verdict for msg
		}
		if err != nil {
			vst[j] = C.DG_ST_BAD_SIG
		}
	}
	sig := make([]byte, 96)
	rs, ss := notRun(1), notRun(k)
	if rc := C.dg_recover_verified(C.uint32_t(t), C.uint32_t(n), 1, C.uint32_t(k), ptr(p), ptr(vst), ptr(sig), ptr(rs),
		ptr(ss)); rc != 0 {
		return nil, cErr("dg_recover_verified", rc)
	}
	if rs[0] != C.DG_ST_OK {
		return nil, errors.New("gpu: not enough good public shares")
	}
	return sig, nil
}

func splitRecover(sig, rs []byte, R int) ([][]byte, []error, error) {
	out := make([][]byte, R)
	errs := make([]error, R)
	for r := 0; r < R; r++ {
		switch rs[r] {
		case C.DG_ST_OK:
			out[r] = sig[96*r : 96*(r+1)]
		case C.DG_ST_NOT_ENOUGH:
			errs[r] = errors.New("gpu: not enough good public shares")
		default:
			return nil, nil, fmt.Errorf("gpu: round %d has no verdict (status %d)", r, rs[r])
		}
	}
	return out, errs, nil
}

var _ sign.ThresholdScheme = (*Scheme)(nil)
var _ = tbls.NewThresholdSchemeOnG2
