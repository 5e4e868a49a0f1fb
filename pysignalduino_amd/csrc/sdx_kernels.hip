// sdx_kernels.hip -- MI355X (gfx950) kernels of the batched SIGNALduino demodulator.
//
// MU / MS engine (k_pulses): one 256-thread workgroup per tile of TM messages.
//   stage    : the tile's pulse strings are read coalesced from HBM once and turned into
//              per-id position bitmaps in LDS (10 ballots per 64 characters).
//   filter   : lane = message, the 4 waves split the class table (bank order) into
//              contiguous quarters; every protocol is wave-uniform, so the bank record is
//              read with scalar loads and the loop structure is uniform.  A lane runs
//              the reference's candidate gates (clock gate, pattern_exists for
//              start/sync/one/zero/float) for its message.
//   decode   : each surviving (message x protocol) pair is decoded by the WHOLE wave
//              (one wavefront per candidate pair): unit bitmaps, stride streams built with
//              ballots, an exact re.finditer emulation, lane-parallel chunk->bit mapping,
//              postDemodulation, padding, hex, modulematch DFA, staged in LDS.
//   flush    : results are written in reference order (message, bank order, match order)
//              with one global atomic per tile for the record/heap space.
// MC engine (k_mc): lane = frame, the 12 clockrange protocols are a uniform loop.
#include "sdx_device.h"
#include "sdx_lane.h"
#include "sdx_mc.h"

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#ifdef SDX_WGTIME
// diagnostic build only (tools/wg_timeline.py): per-workgroup start / end stamps (s_memrealtime, 100 MHz)
__device__ unsigned long long g_wgt[2 * 65536];
#endif
#ifdef SDX_PROF
__device__ unsigned long long g_prof[32];
__device__ unsigned long long g_gprof[2][128];  // per MU clock group / MS protocol: wave-cycles, grabs
#define PROF_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(slot, v)                                                                   \
  do {                                                                                      \
    if (__lane_id() == 0) L.prof[wave][slot] += (unsigned)(__builtin_amdgcn_s_memtime() - (v)); \
  } while (0)
#define PROF_CNT(slot, x)                                                                   \
  do {                                                                                      \
    if (__lane_id() == 0) L.prof[wave][slot] += (unsigned)(x);                              \
  } while (0)
// divergent code: the lowest active lane accounts the wave's time
#define PROF_ADDD(slot, v)                                                                  \
  do {                                                                                      \
    if (__lane_id() == __ffsll((unsigned long long)__builtin_amdgcn_read_exec()) - 1)       \
      L.prof[wave][slot] += (unsigned)(__builtin_amdgcn_s_memtime() - (v));                 \
  } while (0)
// per-lane event count (divergent code)
#define PROF_CNTL(slot) atomicAdd(&L.prof[wave][slot], 1u)
#else
#define PROF_T(v)
#define PROF_ADD(slot, v)
#define PROF_ADDD(slot, v)
#define PROF_CNT(slot, x)
#define PROF_CNTL(slot)
#endif

#ifndef SDX_NO_RAISE_CHECK
#define SDX_NO_RAISE_CHECK 1
#endif

namespace sdx {

constexpr int POOL_REC = 640;    // MU/MS: staged results per tile (shared by the 4 waves)
constexpr int POOL_HEAP = 16384; // MU/MS: staged payload bytes per tile
constexpr int POOL_REC_MS = 256;   // short MS tiles: ~1 result per message; smaller LDS -> more tiles/CU
constexpr int POOL_HEAP_MS = 8192;

struct StageRec {
  uint32_t off;
  uint16_t len, proto;
  uint32_t bitlen;  // bit_length; with STAGE_NIB set: bits 0-15 bit_length, 16-30 the payload's hex digits
  uint8_t msg, wave;
  uint16_t rank;
};
// The finishers build every payload as preamble + digits + postamble of its protocol; when the
// digits are uppercase hex (all but f"{None}"), the record says so, and the flush writes the
// exchange's nibble class (sdx_out.xrec_dev, ABI 12) without reading the payload again
constexpr uint32_t STAGE_NIB = 0x80000000u;
SDX_DEV uint32_t stage_bitlen(int bitlen, int hex_digits, int pre_len) {
  return (hex_digits >= 0 && hex_digits < 32768 && pre_len <= 255 && (uint32_t)bitlen < 65536u)
             ? (STAGE_NIB | ((uint32_t)hex_digits << 16) | (uint32_t)bitlen)
             : (uint32_t)bitlen;
}

// MU (NW <= 4): a (message, protocol) pair that passed the pattern filters, queued for the
// compacted decode (lane = pair)
struct MuItem {
  uint32_t st_lo, st_hi;    // start target string (nibbles)
  uint16_t u0, u1, u2;      // one / zero / float target strings (width <= 4 -> 4 nibbles)
  uint16_t idx, p;          // search start position, protocol index
  uint8_t mi, fmask;        // tile message, found-key mask
};
constexpr int QCAP = 128;  // per-wave ring: < 64 pending before a push of <= 64
#ifndef SDX_LANE_WAVES
#define SDX_LANE_WAVES 8
#endif
constexpr int LANE_WAVES = SDX_LANE_WAVES;  // short variants: 8 waves (512 threads) share one tile

// MS (NW <= 4): a (message, protocol) pair that passed the sync/one/zero/float lookups, queued
// for the lane decode
struct MsItem {
  uint32_t k0_lo, k0_hi;  // sync target string (nibbles)
  uint16_t k1, k2, k3;    // one / zero / float target strings (width <= 4)
  uint16_t start;         // first chunk position (after the sync)
  uint16_t p;             // protocol index
  uint8_t mi, fmask;      // tile message, found-key mask
};
// Per tile (bench corpus: 1.6 survivors per message, ~104 per tile); more -> tile overflow ->
// exact re-run on the long variant.  No decode inside the protocol loop: the loop's state is
// not live across a decode, so nothing is spilled to scratch
constexpr int MS_SURV_CAP = 1024;
constexpr int MS_DESC_LDS = 96;  // MS decode descriptors staged in LDS (the bank has 66 MS ids)
// the fields the MS lane decode reads per survivor (ms_desc builds one from a record)
struct MsDesc {
  int32_t lir_min, lir_max, pad, pre_off, post_off;
  uint16_t pre_len, post_len;
  uint8_t width, klen[4], recon, postdemo, res;
};  // 32 bytes
static_assert(sizeof(MsDesc) == 32, "MsDesc layout");

// MU (NW <= 4): one finditer match, finished after the protocol loop with lane = match
struct MuMatch {
  uint16_t q, k;         // first unit position, number of full units
  uint16_t u0, u1, u2;   // one / zero / float target strings
  uint16_t p;            // protocol index
  uint8_t mi;            // tile message
  uint8_t flags;         // bit0 tail matched, bits1-2 tail symbol, bits3-5 found-key mask
  uint8_t j;             // match index within the (message, protocol) pair
};
constexpr int MATCH_CAP = 768;  // per tile in LDS (bench corpus: mean 290, max 513); more -> the spill region

// Heavy tiles (a grouped message order puts messages with many results together: up to ~2000
// results and ~37 KB of payload per tile on the bench corpus) overflow the LDS pools into a
// per-tile region of the caller's workspace (sdx_out.work_dev), allocated by the first result
// that needs it: matches, staged records and payload bytes.  Only past these does a tile
// overflow (ST_OVF_TILE -> exact re-run).
constexpr uint32_t SPILL_M = 2048, SPILL_R = 2048, SPILL_H = 49152;
constexpr uint32_t SPILL_OFF_R = SPILL_M * 16, SPILL_OFF_H = SPILL_OFF_R + SPILL_R * 16;
constexpr uint32_t SPILL_BYTES = SPILL_OFF_H + SPILL_H;  // 112 KB
constexpr uint32_t SPILL_NONE = 0xFFFFFFFFu, SPILL_PENDING = 0xFFFFFFFEu, SPILL_FULL = 0xFFFFFFFDu;
constexpr uint32_t HEAP_SPILLED = 0x80000000u;  // StageRec.off: payload in the spill region
constexpr uint8_t REC_HOLE = 0xFF;              // StageRec.msg: LDS slot left unused (result spilled)
static_assert(sizeof(MuMatch) == 16, "MuMatch spill layout");

// LM: 0 = wave-cooperative decode (the long variants), 1 = lane-decode MU (NW <= 4: decode
// descriptors, modulematch tables, match list), 2 = lane-decode MS (NW <= 4).  The lane variants
// have no per-wave byte scratch; the MU one keeps the MU decode
// descriptors and modulematch tables staged in LDS
template <int NW, int TM, int LM>
struct TileLds {
  static constexpr int WS = NW;              // words per id bitmap
  static constexpr int MSTRIDE = 10 * NW + 1;  // odd stride: fewer LDS bank conflicts across lanes
  static constexpr int NBITS = 64 * NW + 64;
  struct Wave {
    uint64_t umask[3][NW];
    uint64_t uany[NW];
    uint64_t smask[NW];
    uint64_t stream[NW + 18];
    uint8_t bits[NBITS];
    uint8_t bits2[NBITS];
  };
  uint64_t bm[TM * MSTRIDE];
  uint64_t pairs[TM][2];  // id-pair presence per message: bit 10a+b <=> "ab" occurs
  int32_t nlen[TM];
  uint32_t raise_key[TM];
  uint32_t digit_ok[TM];
  uint32_t cnt[TM];    // staged results per message (atomic; the old value is the record's rank)
  uint32_t rec_base, heap_base, tile_bad, tot_rec;
  uint32_t mbase[TM];
  struct WaveScratch4 {
    Wave w[4];
  };
  struct NoScratch {};
  // per-wave byte scratch: MS and the long MU variant only (the lane-decode MU variant has none)
  typename std::conditional<LM != 0, NoScratch, WaveScratch4>::type wa;
  // short MS tiles (NW <= 4, not the MU lane variant) stage few results; overflow re-runs on the
  // long variant
  static constexpr int PREC = LM == 1 ? 512 : (NW <= 4 ? POOL_REC_MS : POOL_REC);
  static constexpr int PHEAP = LM == 1 ? 10240 : (NW <= 4 ? POOL_HEAP_MS : POOL_HEAP);  // MU bench tiles: <= 8.1 KB
  StageRec rec[PREC];
  alignas(16) uint8_t heap[PHEAP];
  unsigned long long pool_ctr;  // low 32: staged records, high 32: staged heap bytes (one LDS atomic)
  uint32_t spill_base, sp_rec, sp_heap;  // the tile's spill region (SPILL_NONE: none yet) and its fill
  int ovf, next_p;
  int mm_states, nmatch;
  MuMatch mlist[LM == 1 ? MATCH_CAP : 1];
  alignas(16) sdx_mu_desc desc[LM == 1 ? SDX_MUDESC_LDS : 1];
  // the decode queues live only during the protocol loop, the modulematch tables only in the
  // finish phase after it: one region
  union alignas(16) {
    MuItem q[LM == 1 ? LANE_WAVES : 1][LM == 1 ? QCAP : 1];
    uint8_t mmtab[LM == 1 ? SDX_MMTAB_LDS : 16];
  } u;
  // MS survivors of the whole tile, decoded after the protocol loop with lane = survivor
  MsItem slist[LM == 2 ? MS_SURV_CAP : 1];
  int nsurv;
  MsDesc msdesc[LM == 2 ? MS_DESC_LDS : 1];
#ifdef SDX_PROF
  unsigned int prof[LM != 0 ? LANE_WAVES : 4][28];  // s_memtime deltas per wave (< 2^32 per kernel)
#endif
};

SDX_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

SDX_DEV int lanes_below(uint64_t mask) {
  const int l = lane_id();
  return popc64(l ? (mask & ((1ull << l) - 1)) : 0ull);
}

// ---------------------------------------------------------------------------------------------
// staged-result helpers (wave-uniform callers)
// ---------------------------------------------------------------------------------------------
// allocate `total` payload bytes + one record in the tile pool (lane 0 does the LDS atomics);
// returns the heap offset (broadcast to the wave) or -1 when the pool is full
template <class T>
SDX_DEV int pool_alloc(T& L, int total, int* rec_slot) {
  int h = -1, r = -1;
  if (lane_id() == 0) {
    const unsigned long long o = atomicAdd(&L.pool_ctr, ((unsigned long long)total << 32) | 1ull);
    r = (int)(uint32_t)o;
    h = (int)(o >> 32);
    if (r >= T::PREC || h + total > T::PHEAP) {
      L.ovf = 1;
      h = -1;
    }
  }
  h = bcast_i(h, 0);
  *rec_slot = bcast_i(r, 0);
  return h;
}

template <class T>
SDX_DEV void pool_commit(T& L, int slot, int wave, int msg_local, int proto, int off, int total, int bitlen) {
  if (lane_id() == 0) {
    StageRec r;
    r.off = (uint32_t)off;
    r.len = (uint16_t)total;
    r.proto = (uint16_t)proto;
    r.bitlen = (uint32_t)bitlen;
    r.msg = (uint8_t)msg_local;
    r.wave = (uint8_t)wave;
    r.rank = (uint16_t)atomicAdd(&L.cnt[msg_local], 1u);
    L.rec[slot] = r;
  }
  wave_sync();
}

// the tile's spill region in the workspace (allocated once, by the first lane that needs it), or
// SPILL_NONE when the workspace is absent or exhausted
template <class T>
SDX_DEV uint32_t spill_region(T& L, const sdx_out& out) {
  uint32_t b = __hip_atomic_load(&L.spill_base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (b >= SPILL_PENDING) {  // none yet: one leader lane per wave; the first leader allocates, the
                             // others wait for its address (waves progress independently)
    const int leader = ffs64(ballot(true));
    if (lane_id() == leader) {
      uint32_t cur = atomicCAS(&L.spill_base, SPILL_NONE, SPILL_PENDING);
      if (cur == SPILL_NONE) {
        // cursor[3] counts the regions handed out (one per tile at most, so it cannot wrap); a
        // region past the workspace is SPILL_FULL
        const uint32_t idx = atomicAdd(&out.cursor_dev[3], 1u);
        const uint64_t o = (uint64_t)idx * SPILL_BYTES;
        cur = (out.work_dev && o + SPILL_BYTES <= out.work_cap) ? (uint32_t)o : SPILL_FULL;
        __hip_atomic_store(&L.spill_base, cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      while (cur == SPILL_PENDING) cur = __hip_atomic_load(&L.spill_base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      b = cur;
    }
    b = (uint32_t)__shfl((int)b, leader);
  }
  if (b == SPILL_FULL || !out.work_dev || (uint64_t)b + SPILL_BYTES > out.work_cap) return SPILL_NONE;
  return b;
}

// one staged result (lane-level writers): record slot + `span` payload bytes (multiple of 8) in the
// tile's LDS pool, else in its spill region; false (tile overflow) when neither has room
struct PoolSlot {
  StageRec* rec;
  uint8_t* heap;
  uint32_t off;  // StageRec.off
};
template <class T>
SDX_DEV bool pool_take(T& L, const sdx_out& out, int span, PoolSlot* ps) {
  const unsigned long long o = atomicAdd(&L.pool_ctr, ((unsigned long long)span << 32) | 1ull);
  const int slot = (int)(uint32_t)o, off = (int)(o >> 32);
  if (slot < T::PREC && off + span <= T::PHEAP) {
    ps->rec = &L.rec[slot];
    ps->heap = L.heap + off;
    ps->off = (uint32_t)off;
    return true;
  }
  if (slot < T::PREC) L.rec[slot].msg = REC_HOLE;  // skipped by the flush
  const uint32_t base = spill_region(L, out);
  const uint32_t rs = atomicAdd(&L.sp_rec, 1u), hs = atomicAdd(&L.sp_heap, (uint32_t)span);
  if (base == SPILL_NONE || rs >= SPILL_R || hs + (uint32_t)span > SPILL_H) {
    L.ovf = 1;
    return false;
  }
  uint8_t* reg = out.work_dev + base;
  ps->rec = reinterpret_cast<StageRec*>(reg + SPILL_OFF_R) + rs;
  ps->heap = reg + SPILL_OFF_H + hs;
  ps->off = HEAP_SPILLED | hs;
  return true;
}

// copy a bank string to LDS (lanes in parallel)
SDX_DEV void copy_str(uint8_t* dst, const uint8_t* src, int n) {
  for (int i = lane_id(); i < n; i += WAVE) dst[i] = src[i];
}

// bits[0..nb) (values 0/1/2='F') -> dmsg bytes at dst; returns length, or -1 for the 'None'
// (bin_str_2_hex_str -> None, helpers.py:44-45) case.  Wave-cooperative.
SDX_DEV int any_float(const uint8_t* bits, int nb) {
  bool f = false;
  for (int i = lane_id(); i < nb; i += WAVE) f |= bits[i] == 2;
  return ballot(f) != 0;
}

// helpers.py:28-64: nibbles from the right, leading partial nibble kept, uppercase
SDX_DEV int hex_digits(const uint8_t* bits, int nb, uint8_t* dst, int strip_zero) {
  const int nd = (nb + 3) >> 2;
  // digit d (from the left) covers bits [e-4, e) with e = nb - 4*(nd-1-d), clipped at 0
  int skip = 0;
  if (strip_zero) {  // str.lstrip('0')
    skip = nd;
    for (int d0 = 0; d0 < nd; d0 += WAVE) {
      const int d = d0 + lane_id();
      int v = 0;
      if (d < nd) {
        const int e = nb - 4 * (nd - 1 - d), a = (e - 4 > 0) ? e - 4 : 0;
        for (int i = a; i < e; ++i) v = (v << 1) | bits[i];
      }
      const uint64_t nz = ballot(d < nd && v != 0);
      if (nz) {
        skip = d0 + ffs64(nz);
        break;
      }
    }
  }
  for (int d = skip + lane_id(); d < nd; d += WAVE) {
    const int e = nb - 4 * (nd - 1 - d), a = (e - 4 > 0) ? e - 4 : 0;
    int v = 0;
    for (int i = a; i < e; ++i) v = (v << 1) | bits[i];
    dst[d - skip] = (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
  }
  return nd - skip;
}

template <class T>
SDX_DEV void raise_msg(T& L, int msg_local, int proto, int kind) {
  if (lane_id() == 0) atomicMin(&L.raise_key[msg_local], ((uint32_t)proto << 8) | (uint32_t)kind);
  wave_sync();
}

// ---------------------------------------------------------------------------------------------
// MU: finish one match (message_unsynced.py:230-290)
// ---------------------------------------------------------------------------------------------
template <int NW, int TM, int LM>
SDX_DEV void finish_mu(TileLds<NW, TM, LM>& L, int wave, const BankView& bv, const sdx_mu_proto* rec, int p, int s,
                       int nb) {
  auto& W = L.wa.w[wave];
  uint8_t* buf = W.bits;
  PROF_T(t_pd);
  // postDemodulation (:231-250): 'F' -> int() ValueError caught -> bits unchanged
  if (cld(&rec->postdemo) != SDX_PD_NONE && !any_float(buf, nb)) {
    int rc = 0, no = 0;
    if (lane_id() == 0) rc = run_postdemo(cld(&rec->postdemo), buf, nb, W.bits2, &no);
    rc = bcast_i(rc, 0);
    no = bcast_i(no, 0);
    wave_sync();
    if (rc == 0) return;  // rcode < 1 -> match dropped
    if (rc == 1) {
      buf = W.bits2;
      nb = no;
    }  // rc == -1: ValueError inside the method, caught -> bits unchanged
  }
  PROF_ADD(7, t_pd);
  PROF_T(t_fmt);
  // padding (:257-259), after postDemod
  const int pad = cld(&rec->pad_bits);
  int nbp = nb;
  nbp = (nbp + pad - 1) / pad * pad;  // append '0' until len % pad == 0 (pad >= 1, bank.py)
  for (int i = nb + lane_id(); i < nbp; i += WAVE) buf[i] = 0;
  wave_sync();
  const bool isf = any_float(buf, nbp);
  int dlen;
  if (cld(&rec->dispatch_bin)) dlen = nbp;
  else if (isf) {
    if (cld(&rec->remove_zero)) {  // None.lstrip('0') -> AttributeError (:269)
      raise_msg(L, s, p, SDX_RAISE_ATTRIBUTE);
      return;
    }
    dlen = 4;  // f"{None}"
  } else {
    dlen = -2;  // computed below
  }
  // hex digit geometry (helpers.py:28-64) and str.lstrip('0') for remove_zero
  const int nd = (nbp + 3) >> 2;
  int skip = 0;
  if (dlen == -2) {
    if (cld(&rec->remove_zero)) {
      skip = nd;
      for (int d0 = 0; d0 < nd; d0 += WAVE) {
        const int d = d0 + lane_id();
        int v = 0;
        if (d < nd) {
          const int e = nbp - 4 * (nd - 1 - d), a = (e - 4 > 0) ? e - 4 : 0;
          for (int i = a; i < e; ++i) v = (v << 1) | buf[i];
        }
        const uint64_t nz = ballot(d < nd && v != 0);
        if (nz) {
          skip = d0 + ffs64(nz);
          break;
        }
      }
    }
    dlen = nd - skip;
  }
  auto dchar = [&](int d) -> uint8_t {  // character d of dmsg, computed from the bits
    if (cld(&rec->dispatch_bin)) return buf[d] == 2 ? 'F' : (uint8_t)('0' + buf[d]);
    if (isf) return (uint8_t)"None"[d];
    const int dd = d + skip, e = nbp - 4 * (nd - 1 - dd), a = (e - 4 > 0) ? e - 4 : 0;
    int v = 0;
    for (int i = a; i < e; ++i) v = (v << 1) | buf[i];
    return (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
  };
  if (cld(&rec->mm_dfa) >= 0) {  // re.search(modulematch, payload) (:277-280) before staging anything
    int ok = 0;
    if (lane_id() == 0) {
      const sdx_dfa D = bv.dfa[cld(&rec->mm_dfa)];
      const uint8_t* t256 = bv.t256 + D.t256_off;
      const uint8_t* fl = bv.dflags + D.flags_off;
      int st = cld(&rec->mm_pre_state);
      const int tot = dlen + cld(&rec->post_len);
      int i = 0;
      for (; i < tot; ++i) {
        const uint8_t f = fl[st];
        if (f & 5) break;  // accepted or dead
        const uint8_t c = i < dlen ? dchar(i) : bv.str[cld(&rec->post_off) + i - dlen];
        st = t256[st * 256 + c];
      }
      const uint8_t f = fl[st];
      ok = (f & 1) ? 1 : ((f & 4) ? 0 : ((i == tot && (f & 2)) ? 1 : 0));
    }
    PROF_ADD(9, t_fmt);
    if (!bcast_i(ok, 0)) return;
  }
  PROF_T(t_wr);
  const int total = cld(&rec->pre_len) + dlen + cld(&rec->post_len);
  int slot;
  const int off = pool_alloc(L, total, &slot);
  if (off < 0) return;
  uint8_t* dst = L.heap + off;
  copy_str(dst, bv.str + cld(&rec->pre_off), cld(&rec->pre_len));
  for (int d = lane_id(); d < dlen; d += WAVE) dst[cld(&rec->pre_len) + d] = dchar(d);
  copy_str(dst + cld(&rec->pre_len) + dlen, bv.str + cld(&rec->post_off), cld(&rec->post_len));
  pool_commit(L, slot, wave, s, p, off, total, (int)stage_bitlen(nbp, isf ? -1 : dlen, cld(&rec->pre_len)));
  PROF_ADD(8, t_wr);
  PROF_CNT(20, 1);
}

// ---------------------------------------------------------------------------------------------
// MU: decode one surviving (message, protocol) pair with the whole wave
// (message_unsynced.py:146-290; re.finditer emulated exactly)
// ---------------------------------------------------------------------------------------------
template <int NW, int TM, int LM>
SDX_DEV void decode_mu(TileLds<NW, TM, LM>& L, int wave, const BankView& bv, const sdx_mu_proto* rec, int p, int s,
                       int idx, uint64_t st_tgt, uint64_t ut0, uint64_t ut1, uint64_t ut2, int fmask) {
  using T = TileLds<NW, TM, LM>;
  auto& W = L.wa.w[wave];
  const int lane = lane_id();
  const uint64_t* bm = &L.bm[s * T::MSTRIDE];
  const int n = L.nlen[s], nw = (n + 63) >> 6;
  const int Lw = cld(&rec->width);
  const int lenS = cld(&rec->has_start) ? (int)cld(&rec->start.len) : 0;
  const uint64_t ut[3] = {ut0, ut1, ut2};
  const uint8_t SYM[3] = {1, 0, 2};
  PROF_T(t_setup);
  PROF_CNT(21, 1);
  // pattern_lookup: distinct unit strings, value = last writer (:122)
  uint64_t uni[3] = {0, 0, 0};
  uint8_t usym[3] = {0, 0, 0};
  int nu = 0;
  for (int k = 0; k < 3; ++k) {
    if (!((fmask >> k) & 1)) continue;
    int j = 0;
    for (; j < nu; ++j)
      if (uni[j] == ut[k]) break;
    if (j == nu) uni[nu++] = ut[k];
    usym[j] = SYM[k];
  }
  // end_pattern_lookup: pstr[:-1], first writer wins (:124-127); regex tail only with reconstructBit
  uint64_t ek[3] = {0, 0, 0};
  uint8_t esym[3] = {0, 0, 0};
  int ne = 0;
  if (cld(&rec->recon) && Lw > 1) {
    const uint64_t msk = (Lw - 1 >= 16) ? ~0ull : ((1ull << (4 * (Lw - 1))) - 1);
    for (int k = 0; k < 3; ++k) {
      if (!((fmask >> k) & 1)) continue;
      const uint64_t key = ut[k] & msk;
      int j = 0;
      for (; j < ne; ++j)
        if (ek[j] == key) break;
      if (j == ne) {
        ek[ne] = key;
        esym[ne] = SYM[k];
        ++ne;
      }
    }
  }
  // unit / start position bitmaps
  if (lane < nw) {
    uint64_t any = 0;
    for (int j = 0; j < nu; ++j) {
      uint64_t m = ~0ull;
      for (int i = 0; i < Lw; ++i) {
        const int id = (int)((uni[j] >> (4 * i)) & 15), wo = lane + (i >> 6);
        m &= (wo < nw) ? bm_window(bm + id * T::WS, wo, i & 63, nw) : 0ull;
      }
      W.umask[j][lane] = m;
      any |= m;
    }
    W.uany[lane] = any;
    uint64_t sm = ~0ull;
    for (int i = 0; i < lenS; ++i) {
      const int id = (int)((st_tgt >> (4 * i)) & 15), wo = lane + (i >> 6);
      sm &= (wo < nw) ? bm_window(bm + id * T::WS, wo, i & 63, nw) : 0ull;
    }
    W.smask[lane] = sm;
  }
  wave_sync();
  // stride streams: stream r, bit i = a unit starts at position r + i*Lw
  const int nunits = (n + Lw - 1) / Lw;
  const int sw = (nunits + 63) >> 6;
  for (int r = 0; r < Lw; ++r) {
    for (int c = 0; c < sw; ++c) {
      const int x = r + (c * 64 + lane) * Lw;
      const bool b = x < n && ((W.uany[x >> 6] >> (x & 63)) & 1ull);
      const uint64_t bb = ballot(b);
      if (lane == 0) W.stream[r * sw + c] = bb;
    }
  }
  wave_sync();
  auto runlen = [&](int q) -> int {
    const int r = q % Lw, i = q / Lw;
    const uint64_t* S = W.stream + r * sw;
    int k = 0;
    for (int w = i >> 6, b = i & 63; w < sw; ++w, b = 0) {
      const uint64_t x = S[w] >> b;
      const uint64_t inv = ~x;
      const int t = inv ? ffs64(inv) : 64;
      k += t;
      if (t < 64 - b) break;
    }
    return k;
  };
  const int lmin = cld(&rec->length_min);
  int pos = idx;
  PROF_ADD(4, t_setup);
  while (true) {
    PROF_T(t_scan);
    // first s >= pos where START occurs and >= length_min units follow
    int sfound = -1, kfound = 0;
    const int last = n - lenS;
    for (int c = pos >> 6; c <= (last >> 6); ++c) {
      const int sx = c * 64 + lane;
      bool cand = sx >= pos && sx <= last;
      if (cand && lenS > 0) cand = (W.smask[sx >> 6] >> (sx & 63)) & 1ull;
      const int k = cand ? runlen(sx + lenS) : 0;
      const uint64_t bb = ballot(cand && k >= lmin);
      if (bb) {
        const int l = ffs64(bb);
        sfound = c * 64 + l;
        kfound = bcast_i(k, l);
        break;
      }
    }
    PROF_ADD(5, t_scan);
    if (sfound < 0) break;
    PROF_CNT(22, 1);
    const int q = sfound + lenS, e0 = q + kfound * Lw;
    int em = -1;
    for (int j = 0; j < ne; ++j)
      if (match_at(bm, T::WS, n, ek[j], Lw - 1, e0)) {
        em = j;
        break;
      }
    const int G = kfound * Lw + (em >= 0 ? Lw - 1 : 0);
    if (G == 0) {  // chunks == [] -> chunks[-1] IndexError (:212): the whole message raises
      raise_msg(L, s, p, SDX_RAISE_INDEX);
      return;
    }
    pos = q + G;
    const int nchunks = kfound + (em >= 0 ? 1 : 0);
    if (nchunks > cld(&rec->length_max)) continue;  // (:217-218)
    PROF_T(t_bits);
    for (int i = lane; i < kfound; i += WAVE) {
      const int x = q + i * Lw;
      uint8_t sy = 0;
      for (int j = 0; j < nu; ++j)
        if ((W.umask[j][x >> 6] >> (x & 63)) & 1ull) sy = usym[j];
      W.bits[i] = sy;
    }
    if (em >= 0 && lane == 0) W.bits[kfound] = esym[em];
    wave_sync();
    PROF_ADD(6, t_bits);
    finish_mu(L, wave, bv, rec, p, s, nchunks);
    if ((L.raise_key[s] >> 8) <= (uint32_t)p) return;  // this protocol made the message raise
  }
}

// ---------------------------------------------------------------------------------------------
// MU, lane = message (short variant): finish one match (message_unsynced.py:230-290).
// The chunk symbols are not materialised unless a postDemod method needs them: symbol b is
// read from the unit masks at position q + b*Lw (V1: units mapping to '1', VF: to 'F').
// ---------------------------------------------------------------------------------------------
template <int NW>
SDX_DEV M<NW> m_range(int a, int b) {  // positions [a, b)
  M<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int lo = a - 64 * i, hi = b - 64 * i;
    uint64_t w = 0;
    if (hi > 0 && lo < 64) {
      w = ~0ull;
      if (lo > 0) w &= ~0ull << lo;
      if (hi < 64) w &= (hi > 0) ? ((1ull << hi) - 1) : 0ull;
    }
    r.w[i] = w;
  }
  return r;
}

// little-endian byte stream into 8-byte aligned LDS words (the tail word is zero-padded)
struct ByteWriter {
  uint64_t* dst;
  uint64_t acc = 0;
  int n = 0;
  SDX_DEV explicit ByteWriter(uint64_t* d) : dst(d) {}
  // append the low `cnt` (<= 8) bytes of `chunk` (its higher bytes are zero)
  SDX_DEV void put(uint64_t chunk, int cnt) {
    acc |= chunk << (8 * n);
    const uint64_t spill = n ? chunk >> (64 - 8 * n) : 0ull;
    n += cnt;
    if (n >= 8) {
      *dst++ = acc;
      acc = spill;
      n -= 8;
    }
  }
  SDX_DEV void flush() {
    if (n) *dst = acc;
  }
};

// append `len` bytes of a string in global memory: 8 independent byte loads per step, so one
// memory latency per 8 bytes instead of one per byte
SDX_DEV void put_str(ByteWriter& w, const uint8_t* s, int len) {
  for (int i = 0; i < len; i += 8) {
    const int c = len - i < 8 ? len - i : 8;
    uint64_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < c) x |= (uint64_t)s[i + j] << (8 * j);
    w.put(x, c);
  }
}

// 8 hex digits (nibble i of x = digit i) -> 8 ASCII bytes '0'-'9','A'-'F' (byte i); only the low
// `cnt` bytes are kept
SDX_DEV uint64_t hex8(uint64_t x, int cnt) {
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  const uint64_t ge10 = ((x + 0x0606060606060606ull) >> 4) & 0x0101010101010101ull;
  x += 0x3030303030303030ull + ge10 * 7ull;
  return cnt >= 8 ? x : x & ((1ull << (8 * cnt)) - 1);
}

// pattern_lookup (message_unsynced.py:113-123): U = every unit occurrence; V1 / VF = occurrences
// whose symbol is '1' / 'F' (the LAST writer of an identical unit string decides its symbol)
template <int NW>
SDX_DEV void sym_masks(const uint64_t* bm, uint64_t ut0, uint64_t ut1, uint64_t ut2, int fmask, int Lw, M<NW>* U,
                       M<NW>* V1, M<NW>* VF) {
  const uint64_t ut[3] = {ut0, ut1, ut2};
  const uint8_t SYM[3] = {1, 0, 2};
  *U = m_zero<NW>();
  if (V1) *V1 = m_zero<NW>();
  if (VF) *VF = m_zero<NW>();
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {
    if (!((fmask >> kk) & 1)) continue;
    uint8_t fs = SYM[kk];
#pragma unroll
    for (int j = kk + 1; j < 3; ++j)
      if (((fmask >> j) & 1) && ut[j] == ut[kk]) fs = SYM[j];
    const M<NW> occ = m_occ<NW>(bm, ut[kk], Lw);
    *U = m_or(*U, occ);
    if (V1 && fs == 1) *V1 = m_or(*V1, occ);
    if (VF && fs == 2) *VF = m_or(*VF, occ);
  }
}

template <int NW, class T>
SDX_DEV void finish_mu_lane(T& L, const sdx_out& out, int wave, const BankView& bv, const sdx_mu_proto* rec, const sdx_mu_desc& d, int p,
                            int mi, int j,
                            int q, int k, int Lw, bool emf, uint8_t esym, const M<NW>& V1, const M<NW>& VF) {
  constexpr int NB = 64 * NW + 64;
  PROF_T(t_x);
  int nb = k + ((emf && Lw > 1) ? 1 : 0);
  // the chunk symbols as two packed bitstrings: P1 = symbol '1', PF = symbol 'F'
  M<NW> P1 = m_stride_extract(V1, q, Lw, k), PF = m_zero<NW>();
  if (m_any(VF)) PF = m_stride_extract(VF, q, Lw, k);  // most protocols have no float symbol
  if (nb > k) {
    if (esym == 1) m_set(P1, k);
    if (esym == 2) m_set(PF, k);
  }
  bool anyf = m_any(PF);
  PROF_ADDD(6, t_x);
  PROF_T(t_pd);
  uint8_t pout[NB];
  bool usearr = false;
  if (d.postdemo != SDX_PD_NONE && !anyf) {  // 'F' -> int() ValueError caught -> unchanged
    uint8_t pin[NB];
    for (int b = 0; b < nb; ++b) pin[b] = m_test(P1, b) ? 1 : 0;
    int no = 0;
    const int rc = run_postdemo(d.postdemo, pin, nb, pout, &no);
    if (rc == 0) return;  // rcode < 1: match dropped
    if (rc == 1) {
      usearr = true;
      nb = no;
    }
  }
  PROF_ADDD(7, t_pd);
  PROF_T(t_fmt);
  const int pad = d.pad_bits;
  int nbp = nb;
  nbp = (nbp + pad - 1) / pad * pad;  // append '0' until len % pad == 0 (pad >= 1, bank.py)
  const int nd = (nbp + 3) >> 2;
  if (!usearr && 4 * nd > 64 * NW) {  // does not fit the packed words: use the byte array
    for (int b = 0; b < nb; ++b) pout[b] = m_test(PF, b) ? 2 : (m_test(P1, b) ? 1 : 0);
    usearr = true;
  }
  // hex digits (helpers.py:28-64): right-align the bitstring to a nibble boundary and reverse the
  // bits inside each nibble -> nibble d of H is hex digit d
  M<NW> H = m_zero<NW>();
  if (!usearr) {
    H = m_shl_small(P1, 4 * nd - nbp);
#pragma unroll
    for (int i = 0; i < NW; ++i) H.w[i] = nibrev(H.w[i]);
  }
  auto digit = [&](int d) -> int {
    if (!usearr) return (int)((m_word(H, d >> 4) >> (4 * (d & 15))) & 15ull);
    const int e = nbp - 4 * (nd - 1 - d), a = (e - 4 > 0) ? e - 4 : 0;
    int v = 0;
    for (int i = a; i < e; ++i) v = (v << 1) | (i < nb ? pout[i] : 0);
    return v;
  };
  const bool binm = d.dispatch_bin != 0;
  // fast path: plain hex digits straight from the nibble-reversed words H
  const bool fast = !usearr && !anyf && !binm;
  int dlen, skip = 0;
  if (binm) {
    dlen = nbp;
  } else if (anyf) {
    if (d.remove_zero) {  // None.lstrip('0') -> AttributeError (:269)
      atomicMin(&L.raise_key[mi], ((uint32_t)p << 8) | SDX_RAISE_ATTRIBUTE);
      return;
    }
    dlen = 4;
  } else {
    if (d.remove_zero) {
      if (fast) {  // first non-zero nibble (H holds no bits past digit nd)
        const int f = m_first(H, 0);
        skip = (f < 0 || (f >> 2) >= nd) ? nd : (f >> 2);
      } else {
        while (skip < nd && digit(skip) == 0) ++skip;
      }
    }
    dlen = nd - skip;
  }
  auto dchar = [&](int i) -> uint8_t {
    if (binm) {
      if (usearr) return (uint8_t)(i < nb ? (pout[i] == 2 ? 'F' : '0' + pout[i]) : '0');
      return m_test(PF, i) ? 'F' : (uint8_t)('0' + (m_test(P1, i) ? 1 : 0));
    }
    if (anyf) return (uint8_t)"None"[i];
    const int v = digit(i + skip);
    return (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
  };
  const int pre_len = d.pre_len, post_len = d.post_len;
  const uint8_t* pre_g = pre_len > 16 ? bv.str + cld(&rec->pre_off) : nullptr;     // long strings: heap
  const uint8_t* post_g = post_len > 2 ? bv.str + cld(&rec->post_off) : nullptr;
  uint64_t pre0, pre1;  // the inline strings as words (no dynamic indexing into the descriptor)
  __builtin_memcpy(&pre0, d.pre, 8);
  __builtin_memcpy(&pre1, d.pre + 8, 8);
  const uint64_t post16 = (uint64_t)d.post[0] | ((uint64_t)d.post[1] << 8);
  auto post_c = [&](int i) -> uint8_t { return post_g ? post_g[i] : (uint8_t)(post16 >> (8 * i)); };
  if (d.mm_on == 3 && fast && dlen <= 64) {  // re.search(modulematch, payload) (:277-280): a digit-count
    if (dlen < (int)d.res[0] || dlen > (int)d.res[1]) return;  // interval (bank.py _mm_length_interval)
  } else if ((d.mm_on == 1 || d.mm_on == 3) && fast) {  // re.search(modulematch, payload) (:277-280) on the LDS hex tables
    const uint8_t* hx = L.u.mmtab + 16 * (int)d.mm_base;
    int st = d.pre_state;
    uint64_t cur = 0;
    for (int i = 0; i < dlen; ++i) {
      const int dd = skip + i;
      if (i == 0 || (dd & 15) == 0) cur = m_word(H, dd >> 4) >> (4 * (dd & 15));
      st = hx[16 * st + (int)(cur & 15ull)];
      cur >>= 4;
    }
    st = L.u.mmtab[17 * L.mm_states + d.mm_post + st];
    const uint8_t f = L.u.mmtab[16 * L.mm_states + d.mm_base + st];
    if (!((f & 1) || (!(f & 4) && (f & 2)))) return;
  } else if (d.mm_on) {  // byte walk through the blob's t256 table
    const sdx_dfa D = bv.dfa[cld(&rec->mm_dfa)];
    const uint8_t* t256 = bv.t256 + D.t256_off;
    const uint8_t* fl = bv.dflags + D.flags_off;
    int st = d.pre_state;
    const int tot = dlen + post_len;
    int i = 0;
    for (; i < tot; ++i) {
      if (fl[st] & 5) break;
      const uint8_t c = i < dlen ? dchar(i) : post_c(i - dlen);
      st = t256[st * 256 + c];
    }
    const uint8_t f = fl[st];
    if (!((f & 1) || (!(f & 4) && i == tot && (f & 2)))) return;
  }
  PROF_ADDD(9, t_fmt);
  PROF_T(t_wr);
  // payload (:271-274): preamble + digits + postamble into an 8-byte aligned pool slot
  const int total = pre_len + dlen + post_len;
  const int span = (total + 7) & ~7;
  PoolSlot ps;
  if (!pool_take(L, out, span, &ps)) return;
  ByteWriter w(reinterpret_cast<uint64_t*>(ps.heap));
  if (pre_g) {
    put_str(w, pre_g, pre_len);
  } else {
    auto lowb = [](uint64_t x, int c) { return c >= 8 ? x : x & ((1ull << (8 * c)) - 1); };
    if (pre_len) w.put(lowb(pre0, pre_len), pre_len < 8 ? pre_len : 8);
    if (pre_len > 8) w.put(lowb(pre1, pre_len - 8), pre_len - 8);
  }
  if (fast) {
    for (int t = 0; t < dlen; t += 8) {  // 8 digits per step: nibbles -> bytes -> ASCII hex
      const int b = 4 * (skip + t), wi = b >> 6, sh = b & 63;
      uint64_t x = m_word(H, wi) >> sh;
      if (sh > 32) x |= m_word(H, wi + 1) << (64 - sh);
      const int cnt = (dlen - t < 8) ? dlen - t : 8;
      w.put(hex8(x & 0xFFFFFFFFull, cnt), cnt);
    }
  } else {
    for (int i = 0; i < dlen; ++i) w.put(dchar(i), 1);
  }
  if (post_g) {
    put_str(w, post_g, post_len);
  } else if (post_len) {
    w.put(post_len == 1 ? (post16 & 0xFFull) : post16, post_len);
  }
  w.flush();
  StageRec r;
  r.off = ps.off;
  r.len = (uint16_t)total;
  r.proto = (uint16_t)p;
  r.bitlen = stage_bitlen(nbp, anyf ? -1 : dlen, pre_len);
  r.msg = (uint8_t)mi;
  r.wave = (uint8_t)wave;
  r.rank = (uint16_t)j;  // match index within this (message, protocol) pair: monotone
  PROF_CNTL(20);
  *ps.rec = r;
  PROF_ADDD(8, t_wr);
}

// MU, lane = message: exact re.finditer emulation on register bitmasks (message_unsynced.py:146-290)
template <int NW, class T>
SDX_DEV void decode_mu_lane(T& L, const sdx_out& out, int wave, const BankView& bv, const sdx_mu_proto* rec, const sdx_mu_desc& d, int p,
                            int mi, const uint64_t* bm, int n, int idx, uint64_t st_tgt, uint64_t ut0, uint64_t ut1,
                            uint64_t ut2, int fmask) {
  PROF_T(t_setup);
  const int Lw = d.width;
  const int lenS = d.len_s;
  const uint64_t ut[3] = {ut0, ut1, ut2};
  const uint8_t SYM[3] = {1, 0, 2};
  M<NW> U;
  sym_masks<NW>(bm, ut0, ut1, ut2, fmask, Lw, &U, nullptr, nullptr);
  // end_pattern_lookup: pstr[:-1], first writer wins (:124-127); regex tail only with reconstructBit
  // (kept per source key kk: key kk is live iff found and no earlier found key has the same
  //  prefix -- first writer wins -- which is the insertion-ordered dict without dynamic indexing)
  bool elive[3] = {false, false, false};
  uint64_t ekey[3] = {0, 0, 0};
  if (d.recon && Lw > 1) {
    const uint64_t msk = (Lw - 1 >= 16) ? ~0ull : ((1ull << (4 * (Lw - 1))) - 1);
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      ekey[kk] = ut[kk] & msk;
      bool seen = false;
#pragma unroll
      for (int j = 0; j < kk; ++j) seen |= elive[j] && ekey[j] == ekey[kk];
      elive[kk] = ((fmask >> kk) & 1) && !seen;
    }
  }
  const M<NW> S = lenS ? m_occ<NW>(bm, st_tgt, lenS) : m_all<NW>();
  const int lmin = d.lmin;
  // s: START at s and >= length_min units at s+lenS (with length_min 0 every START qualifies,
  // including one that ends exactly at the end of the data: empty group -> IndexError)
  const M<NW> V = lmin > 0 ? m_and(S, m_shr(m_runs(U, lmin, Lw), lenS)) : S;
  const M<NW> NU = m_not(U);
  int pos = idx, nfin = 0;
  PROF_ADDD(4, t_setup);
  while (true) {
    PROF_T(t_scan);
    const int s = m_first(V, pos);
    if (s < 0 || s > n) break;
    const int q = s + lenS;
    M<NW> Z = NU;
    const uint64_t rw = residue_word(Lw, q % Lw);
#pragma unroll
    for (int i = 0; i < NW; ++i) Z.w[i] &= rw;
    int z = m_first(Z, q);
    if (z < 0) z = q + Lw * ((64 * NW - q + Lw - 1) / Lw);
    const int k = (z - q) / Lw;
    const int e0 = q + k * Lw;
    // the regex tail (?:E1|E2|..)? : first end key (insertion order) that matches at e0
    bool emf = false;
    uint8_t esym = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (!emf && elive[j] && match_at(bm, NW, n, ekey[j], Lw - 1, e0)) {
        emf = true;
        esym = SYM[j];
      }
    }
    const int G = k * Lw + (emf ? Lw - 1 : 0);
    if (G == 0) {  // chunks == [] -> chunks[-1] IndexError (:212)
      atomicMin(&L.raise_key[mi], ((uint32_t)p << 8) | SDX_RAISE_INDEX);
      return;
    }
    pos = q + G;
    const int nch = k + (emf ? 1 : 0);
    PROF_ADDD(5, t_scan);
    if (nch > (int)d.lmax) continue;  // (:217-218); 65535 = none
    PROF_CNTL(22);
    const int slot = atomicAdd(&L.nmatch, 1);  // finished after the protocol loop, lane = match
    MuMatch* dst;
    if (slot < MATCH_CAP) {
      dst = &L.mlist[slot];
    } else {  // heavy tile: the spill region
      const uint32_t base = spill_region(L, out);
      if (base == SPILL_NONE || slot >= MATCH_CAP + (int)SPILL_M) {
        L.ovf = 1;
        return;
      }
      dst = reinterpret_cast<MuMatch*>(out.work_dev + base) + (slot - MATCH_CAP);
    }
    MuMatch mm;
    mm.q = (uint16_t)q;
    mm.k = (uint16_t)k;
    mm.u0 = (uint16_t)ut0;
    mm.u1 = (uint16_t)ut1;
    mm.u2 = (uint16_t)ut2;
    mm.mi = (uint8_t)mi;
    mm.p = (uint16_t)p;
    mm.flags = (uint8_t)((emf ? 1 : 0) | (esym << 1) | (fmask << 3));
    mm.j = (uint8_t)(nfin < 255 ? nfin : 255);
    ++nfin;
    *dst = mm;
  }
}

// ---------------------------------------------------------------------------------------------
// MS: finish (message_synced.py:191-241)
// ---------------------------------------------------------------------------------------------
template <int NW, int TM, int LM>
SDX_DEV void finish_ms(TileLds<NW, TM, LM>& L, int wave, const BankView& bv, const sdx_ms_proto* rec, int p, int s,
                       int nb) {
  auto& W = L.wa.w[wave];
  uint8_t* buf = W.bits;
  if (nb == 0) return;                                      // (:191-192)
  if (cld(&rec->lir_min) != -1 && nb < cld(&rec->lir_min)) return;      // length_in_range (:194-196)
  if (nb > cld(&rec->lir_max)) return;
  int nbp = nb;                                             // padding BEFORE postDemod (:198-200)
  while (nbp % cld(&rec->pad_bits)) ++nbp;
  for (int i = nb + lane_id(); i < nbp; i += WAVE) buf[i] = 0;
  wave_sync();
  nb = nbp;
  if (cld(&rec->postdemo) != SDX_PD_NONE) {                       // no try: 'F' -> ValueError (:209)
    if (any_float(buf, nb)) {
      raise_msg(L, s, p, SDX_RAISE_VALUE);
      return;
    }
    int rc = 0, no = 0;
    if (lane_id() == 0) rc = run_postdemo(cld(&rec->postdemo), buf, nb, W.bits2, &no);
    rc = bcast_i(rc, 0);
    no = bcast_i(no, 0);
    wave_sync();
    if (rc == -1) {
      raise_msg(L, s, p, SDX_RAISE_VALUE);
      return;
    }
    if (rc == 0) return;
    if (no > 0) {
      buf = W.bits2;
      nb = no;
    }
  }
  if (any_float(buf, nb)) return;  // bin_str_2_hex_str -> None -> skipped (:224-226)
  const int dl = (nb + 3) / 4;
  const int total = cld(&rec->pre_len) + dl + cld(&rec->post_len);
  int slot;
  const int off = pool_alloc(L, total, &slot);
  if (off < 0) return;
  uint8_t* dst = L.heap + off;
  copy_str(dst, bv.str + cld(&rec->pre_off), cld(&rec->pre_len));
  hex_digits(buf, nb, dst + cld(&rec->pre_len), 0);
  copy_str(dst + cld(&rec->pre_len) + dl, bv.str + cld(&rec->post_off), cld(&rec->post_len));
  wave_sync();
  pool_commit(L, slot, wave, s, p, off, total, (int)stage_bitlen(nb, dl, cld(&rec->pre_len)));
}

// MS decode loop (:172-189) for one surviving pair, wave-cooperative over chunks
template <int NW, int TM, int LM>
SDX_DEV void decode_ms(TileLds<NW, TM, LM>& L, int wave, const BankView& bv, const sdx_ms_proto* rec, int p, int s,
                       int start, uint64_t k0, uint64_t k1, uint64_t k2, uint64_t k3, int fmask) {
  using T = TileLds<NW, TM, LM>;
  auto& W = L.wa.w[wave];
  const int lane = lane_id();
  const uint64_t* bm = &L.bm[s * T::MSTRIDE];
  const int n = L.nlen[s];
  const int Wd = cld(&rec->width);
  PROF_T(t_msd);
  PROF_CNT(23, 1);
  const uint64_t kt[4] = {k0, k1, k2, k3};
  const int klen[4] = {cld(&rec->key[0].len), cld(&rec->key[1].len), cld(&rec->key[2].len), cld(&rec->key[3].len)};
  const uint8_t KSYM[4] = {3, 1, 0, 2};  // 3 = '' (sync: no bit)
  // pattern_lookup with dict semantics: distinct (string) keys, value = last writer
  uint64_t kk[4];
  int kl[4];
  uint8_t ks[4];
  int nk = 0;
  for (int k = 0; k < 4; ++k) {
    if (!((fmask >> k) & 1)) continue;
    int j = 0;
    for (; j < nk; ++j)
      if (kk[j] == kt[k] && kl[j] == klen[k]) break;
    if (j == nk) {
      kk[nk] = kt[k];
      kl[nk] = klen[k];
      ++nk;
    }
    ks[j] = KSYM[k];
  }
  // end_pattern_lookup: reset after sync, then one/zero/float pstr[:-1], first wins
  uint64_t ek[3];
  uint8_t es[3];
  int ne = 0;
  const int el = Wd - 1;
  const uint64_t emsk = (el >= 16) ? ~0ull : ((1ull << (4 * el)) - 1);
  for (int k = 1; k < 4; ++k) {
    if (!((fmask >> k) & 1) || klen[k] < 1) continue;
    const uint64_t key = kt[k] & emsk;
    const int kel = klen[k] - 1;
    if (kel != el) continue;  // unit lengths equal the width in every modelled bank
    int j = 0;
    for (; j < ne; ++j)
      if (ek[j] == key) break;
    if (j == ne) {
      ek[ne] = key;
      es[ne] = KSYM[k];
      ++ne;
    }
  }
  const bool recon = cld(&rec->recon) != 0;
  const int nch = (start < n) ? (n - start + Wd - 1) / Wd : 0;
  int nb = 0;
  for (int c0 = 0; c0 < nch; c0 += WAVE) {
    const int i = c0 + lane;
    const bool valid = i < nch;
    int cls = -1;  // -1 break, 0..2 bit, 3 skip
    if (valid) {
      const int x = start + i * Wd;
      const int cl = (n - x < Wd) ? n - x : Wd;
      for (int j = 0; j < nk && cls < 0; ++j)
        if (kl[j] == cl && match_at(bm, T::WS, n, kk[j], cl, x)) cls = ks[j];
      if (cls < 0 && recon) {
        const int tl = (cl == Wd) ? cl - 1 : cl;  // chunk[:-1] if full else chunk
        if (tl == el)
          for (int j = 0; j < ne && cls < 0; ++j)
            if (match_at(bm, T::WS, n, ek[j], el, x)) cls = es[j];
      }
    }
    const uint64_t brk = ballot(valid && cls < 0);
    const int lim = brk ? ffs64(brk) : WAVE;
    const bool emit = valid && lane < lim && cls >= 0 && cls != 3;
    const uint64_t em = ballot(emit);
    if (emit) W.bits[nb + lanes_below(em)] = (uint8_t)cls;
    nb += popc64(em);
    if (brk) break;
  }
  wave_sync();
  PROF_ADD(10, t_msd);
  PROF_T(t_msf);
  finish_ms(L, wave, bv, rec, p, s, nb);
  PROF_ADD(11, t_msf);
}

// ---------------------------------------------------------------------------------------------
// MS, lane = (message, protocol) survivor (message_synced.py:160-241) on register bitmasks
// ---------------------------------------------------------------------------------------------
// the fields the MS lane decode reads per survivor, staged in LDS once per tile (the first
// MS_DESC_LDS protocols): the survivors of a tile mix protocols, so reading them from the record
// would be per-lane vector loads from L2 on every decode
SDX_DEV MsDesc ms_desc(const sdx_ms_proto* rec) {
  MsDesc d;
  d.lir_min = cld(&rec->lir_min);
  d.lir_max = cld(&rec->lir_max);
  d.pad = cld(&rec->pad_bits);
  d.pre_off = cld(&rec->pre_off);
  d.post_off = cld(&rec->post_off);
  d.pre_len = (uint16_t)cld(&rec->pre_len);
  d.post_len = (uint16_t)cld(&rec->post_len);
  d.width = (uint8_t)cld(&rec->width);
#pragma unroll
  for (int k = 0; k < 4; ++k) d.klen[k] = (uint8_t)cld(&rec->key[k].len);
  d.recon = (uint8_t)(cld(&rec->recon) != 0);
  d.postdemo = (uint8_t)cld(&rec->postdemo);
  d.res = 0;
  return d;
}

// finish one MS result from its packed bits (P1 = '1', PF = 'F', nb bits): length_in_range,
// padding BEFORE postDemod, postDemod without try, hex (None -> skipped), payload
template <int NW, class T>
SDX_DEV void finish_ms_lane(T& L, const sdx_out& out, const BankView& bv, const MsDesc& D, int p, int mi, const M<NW>& P1,
                            const M<NW>& PF, int nb) {
  constexpr int NB = 64 * NW + 64;
  const int lir_min = D.lir_min, lir_max = D.lir_max, pad = D.pad;
  const int pd = D.postdemo;
  const int pre_len = D.pre_len, post_len = D.post_len;
  const int pre_off = D.pre_off, post_off = D.post_off;
  if (nb == 0) return;  // (:191-192)
  if (lir_min != -1 && nb < lir_min) return;  // length_in_range (:194-196)
  if (nb > lir_max) return;
  int nbits = nb;  // padding (:198-200): appended '0' bits (P1/PF hold zeros beyond nb)
  nbits = (nbits + pad - 1) / pad * pad;  // pad >= 1 (bank.py)
  const bool anyf = m_any(PF);
  uint8_t pout[NB];
  bool usearr = false;
  if (pd != SDX_PD_NONE) {  // (:203-219)
    if (anyf) {  // int('F') -> ValueError, not caught
      atomicMin(&L.raise_key[mi], ((uint32_t)p << 8) | SDX_RAISE_VALUE);
      return;
    }
    uint8_t pin[NB];
    for (int b = 0; b < nbits; ++b) pin[b] = m_test(P1, b) ? 1 : 0;
    int no = 0;
    const int rc = run_postdemo(pd, pin, nbits, pout, &no);
    if (rc == -1) {
      atomicMin(&L.raise_key[mi], ((uint32_t)p << 8) | SDX_RAISE_VALUE);
      return;
    }
    if (rc == 0) return;
    if (no > 0) {  // `if ret:` keeps the bits for an empty list
      usearr = true;
      nbits = no;
    }
  }
  if (!usearr && anyf) return;  // bin_str_2_hex_str -> None -> skipped (:224-226)
  const int nd = (nbits + 3) >> 2;
  if (!usearr && 4 * nd > 64 * NW) {
    for (int b = 0; b < nbits; ++b) pout[b] = m_test(P1, b) ? 1 : 0;
    usearr = true;
  }
  M<NW> H = m_zero<NW>();  // hex digits: right-aligned to a nibble boundary, nibble-reversed
  if (!usearr) {
    H = m_shl_small(P1, 4 * nd - nbits);
#pragma unroll
    for (int i = 0; i < NW; ++i) H.w[i] = nibrev(H.w[i]);
  }
  const uint8_t* pre = bv.str + pre_off;
  const uint8_t* post = bv.str + post_off;
  const int total = pre_len + nd + post_len;
  const int span = (total + 7) & ~7;
  PoolSlot ps;
  if (!pool_take(L, out, span, &ps)) return;
  ByteWriter w(reinterpret_cast<uint64_t*>(ps.heap));
  put_str(w, pre, pre_len);
  if (!usearr) {
    for (int t = 0; t < nd; t += 8) {
      const int b = 4 * t, wi = b >> 6, sh = b & 63;
      uint64_t x = m_word(H, wi) >> sh;
      if (sh > 32) x |= m_word(H, wi + 1) << (64 - sh);
      const int cnt = (nd - t < 8) ? nd - t : 8;
      w.put(hex8(x & 0xFFFFFFFFull, cnt), cnt);
    }
  } else {
    for (int d = 0; d < nd; ++d) {  // nibbles from the right (helpers.py:28-64)
      const int e = nbits - 4 * (nd - 1 - d), a = (e - 4 > 0) ? e - 4 : 0;
      int v = 0;
      for (int i = a; i < e; ++i) v = (v << 1) | pout[i];
      w.put((uint64_t)(v < 10 ? '0' + v : 'A' + v - 10), 1);
    }
  }
  put_str(w, post, post_len);
  w.flush();
  StageRec r;
  r.off = ps.off;
  r.len = (uint16_t)total;
  r.proto = (uint16_t)p;
  r.bitlen = stage_bitlen(nbits, nd, pre_len);
  r.msg = (uint8_t)mi;
  r.wave = 0;
  r.rank = 0;  // one result per (message, protocol)
  *ps.rec = r;
}

template <int NW, class T>
SDX_DEV void decode_ms_lane(T& L, const sdx_out& out, const BankView& bv, const MsDesc& D, int p, int mi, const uint64_t* bm,
                            int n, int start, uint64_t k0, uint64_t k1, uint64_t k2, uint64_t k3, int fmask) {
  const int Wd = D.width;
  const uint64_t kt[4] = {k0, k1, k2, k3};
  const int klen[4] = {D.klen[0], D.klen[1], D.klen[2], D.klen[3]};
  const bool recon = D.recon != 0 && Wd > 1;
  const uint8_t KSYM[4] = {3, 1, 0, 2};  // 3: the sync symbol '' (no bit)
  const int span = start < n ? n - start : 0;
  const int nfull = span / Wd, part = span - nfull * Wd;
  // The chunk loop (:174-189) reads chunk t at position start + t*Wd.  Everything is kept in the
  // position domain (bit p = a key occurrence starting at p), where "chunk t is a unit" is bit
  // start + t*Wd: the break is found there directly, and only the symbol-'1' mask (and, when
  // present, 'F' / sync-in-data) is compacted to chunk order -- one stride extraction instead of
  // one per key.  Wd is 1, 2 or 4 (m_stride_extract, residue_word).
  M<NW> R1 = m_zero<NW>(), RF = m_zero<NW>(), RS = m_zero<NW>(), RU = m_zero<NW>(), RT = m_zero<NW>();
  // pattern_lookup (:122-135): distinct strings, value = the last writer's symbol
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    if (!((fmask >> kk) & 1) || klen[kk] != Wd) continue;
    bool later = false;
#pragma unroll
    for (int j = kk + 1; j < 4; ++j) later |= ((fmask >> j) & 1) && klen[j] == klen[kk] && kt[j] == kt[kk];
    if (later) continue;
    const M<NW> O = m_occ<NW>(bm, kt[kk], Wd);
    RU = m_or(RU, O);
    if (KSYM[kk] == 1) R1 = m_or(R1, O);
    if (KSYM[kk] == 2) RF = m_or(RF, O);
    if (KSYM[kk] == 3) RS = m_or(RS, O);
  }
  // end_pattern_lookup (:124-127, reset after the sync :158): one/zero/float pstr[:-1], first
  // writer wins; a full chunk that is no unit continues with chunk[:-1]'s symbol (:183-187)
  const uint64_t emsk = (Wd - 1 >= 16) ? ~0ull : ((1ull << (4 * (Wd - 1))) - 1);
  if (recon) {
    const M<NW> notU = m_not(RU);
#pragma unroll
    for (int kk = 1; kk < 4; ++kk) {
      if (!((fmask >> kk) & 1) || klen[kk] != Wd) continue;
      const uint64_t key = kt[kk] & emsk;
      bool earlier = false;
#pragma unroll
      for (int j = 1; j < kk; ++j) earlier |= ((fmask >> j) & 1) && klen[j] == Wd && (kt[j] & emsk) == key;
      if (earlier) continue;
      const M<NW> X = m_and(m_occ<NW>(bm, key, Wd - 1), notU);
      RT = m_or(RT, X);
      if (KSYM[kk] == 1) R1 = m_or(R1, X);
      if (KSYM[kk] == 2) RF = m_or(RF, X);
    }
  }
  // chunk grid: positions start + t*Wd, t < nfull
  const int wsh = __ffs(Wd) - 1;
  const uint64_t res = residue_word(Wd, start & (Wd - 1));
  M<NW> G = m_and(m_range_lo<NW>(start + nfull * Wd), m_not(m_range_lo<NW>(start)));
#pragma unroll
  for (int i = 0; i < NW; ++i) G.w[i] &= res;
  // the first chunk that is neither ends the loop (:188-189)
  const int pb = m_first(m_and(G, m_not(m_or(RU, RT))), 0);
  const int k = pb < 0 ? nfull : (pb - start) >> wsh;
  // a partial last chunk: a unit of its length (last writer), else (recon) the chunk as a tail key
  int extra = -1;
  if (k == nfull && part > 0) {
    const int x = start + nfull * Wd;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      if (((fmask >> kk) & 1) && klen[kk] == part && match_at(bm, NW, n, kt[kk], part, x)) extra = KSYM[kk];
    if (extra < 0 && recon && part == Wd - 1) {
#pragma unroll
      for (int kk = 1; kk < 4; ++kk)
        if (extra < 0 && ((fmask >> kk) & 1) && klen[kk] == Wd && match_at(bm, NW, n, kt[kk] & emsk, part, x))
          extra = KSYM[kk];
    }
  }
  // bits = chunks [0, k) without the sync-symbol ones, then the partial chunk's bit
  const M<NW> Gk = m_and(G, m_range_lo<NW>(start + k * Wd));
  M<NW> P1, PF = m_zero<NW>();
  int nb;
  if (!m_any(m_and(RS, Gk))) {
    P1 = m_stride_extract(R1, start, Wd, k);
    if (m_any(m_and(RF, Gk))) PF = m_stride_extract(RF, start, Wd, k);
    nb = k;
  } else {  // a sync-string chunk inside the data (rare): compact serially
    const M<NW> C1 = m_stride_extract(R1, start, Wd, k), CF = m_stride_extract(RF, start, Wd, k),
                CS = m_stride_extract(RS, start, Wd, k);
    P1 = m_zero<NW>();
    nb = 0;
    for (int t = 0; t < k; ++t) {
      if (m_test(CS, t)) continue;
      if (m_test(C1, t)) m_set(P1, nb);
      if (m_test(CF, t)) m_set(PF, nb);
      ++nb;
    }
  }
  if (extra >= 0 && extra != 3) {
    if (extra == 1) m_set(P1, nb);
    if (extra == 2) m_set(PF, nb);
    ++nb;
  }
  finish_ms_lane<NW>(L, out, bv, D, p, mi, P1, PF, nb);
}

// ---------------------------------------------------------------------------------------------
// tile flush: records in (message, protocol, match) order, one atomic per tile.
// Records reach the pool in any order (waves and drained (message, protocol) items run
// concurrently); a record's place inside its message is the number of records of the same
// message with a smaller (protocol, rank) key -- rank is the per-message atomic counter, which
// increases monotonically along one (message, protocol) pair's finditer loop.
// ---------------------------------------------------------------------------------------------
// The exchange's wire form of one payload (include/sdx.h ABI 12, sdx_out.xrec_dev): preamble + D
// uppercase hex digits + postamble of its protocol (message_unsynced.py:271-274,
// message_synced.py:228-229, manchester.py:131-132) -> the xrec word SDX_XREC_NIB | npre << 16 | D,
// else 0 (raw).  The same rule as sdx_exchange.hip nib_digits; run by the flushes on the staged
// payloads (LDS or spill region), so the exchange never re-reads a payload to classify it.
SDX_DEV bool uhex_c(uint8_t c) { return (uint8_t)(c - '0') < 10u || (uint8_t)(c - 'A') < 6u; }
SDX_DEV uint32_t wire_class(const BankView& bv, int kind, int proto, const uint8_t* p, int len) {
  int po, pl, qo = 0, ql = 0;
  if (kind == SDX_KIND_MU) {
    const sdx_mu_proto* r = bv.mu + proto;
    po = r->pre_off, pl = r->pre_len, qo = r->post_off, ql = r->post_len;
  } else if (kind == SDX_KIND_MS) {
    const sdx_ms_proto* r = bv.ms + proto;
    po = r->pre_off, pl = r->pre_len, qo = r->post_off, ql = r->post_len;
  } else {
    const sdx_mc_proto* r = bv.mc + proto;
    po = r->pre_off, pl = r->pre_len;
  }
  if (pl < 0 || ql < 0 || pl > 255 || len < pl + ql) return 0u;
  const int d = len - pl - ql;
  bool ok = true;
  for (int i = 0; i < pl; ++i) ok &= p[i] == bv.str[po + i];
  for (int i = 0; i < ql; ++i) ok &= p[pl + d + i] == bv.str[qo + i];
  for (int i = 0; i < d; ++i) ok &= uhex_c(p[pl + i]);
  return ok ? (SDX_XREC_NIB | ((uint32_t)pl << 16) | (uint32_t)d) : 0u;
}
SDX_DEV uint32_t wire_bytes_x(uint32_t xr, int len) {
  return (xr & SDX_XREC_NIB) ? ((xr & 0xFFFFu) + 1u) >> 1 : (uint32_t)len;
}

template <int NW, int TM, int LM>
SDX_DEV void flush_tile(TileLds<NW, TM, LM>& L, const int* msg_of, int nvalid, const sdx_out& out, const BankView& bv,
                        int kind) {
  using T = TileLds<NW, TM, LM>;
  const int tid = threadIdx.x;
  // staged records: the LDS pool [0, nr_l), then (lane writers of heavy tiles) the spill region
  // [nr_l, nr); payload bytes likewise (StageRec.off with HEAP_SPILLED: spill region)
  constexpr int RMAX = T::PREC + (LM != 0 ? (int)SPILL_R : 0);
  // flush scratch aliases the id bitmaps (dead once every wave has left the protocol loop)
  static_assert(sizeof(L.bm) >= TM * 16 + RMAX * 2, "flush scratch does not fit the bitmaps");
  uint64_t* wsum = reinterpret_cast<uint64_t*>(L.bm);       // per message: payload << 32 | wire bytes
  uint32_t* fill = reinterpret_cast<uint32_t*>(wsum + TM);  // bucket fill per message
  uint32_t* cntm = fill + TM;                               // staged records per message
  uint16_t* bidx = reinterpret_cast<uint16_t*>(cntm + TM);  // record indices bucketed by message
  const bool wx = out.wire_dev != nullptr;                  // the exchange's counts (ABI 12)
  if (tid < TM) {
    fill[tid] = 0;
    cntm[tid] = 0;
    wsum[tid] = 0;
  }
  __syncthreads();
  const int nr_l = (int)(uint32_t)L.pool_ctr < T::PREC ? (int)(uint32_t)L.pool_ctr : T::PREC;
  const int nh_raw = (int)(L.pool_ctr >> 32);
  const int nh_l = nh_raw < T::PHEAP ? nh_raw : T::PHEAP;
  const bool spill = LM != 0 && L.spill_base < SPILL_PENDING;
  const int nr_s = spill ? ((int)L.sp_rec < (int)SPILL_R ? (int)L.sp_rec : (int)SPILL_R) : 0;
  const int nh_s = spill ? ((int)L.sp_heap < (int)SPILL_H ? (int)L.sp_heap : (int)SPILL_H) : 0;
  const int nr = nr_l + nr_s;
  const uint8_t* sreg = spill ? out.work_dev + L.spill_base : nullptr;
  auto rec_at = [&](int i) -> StageRec {
    return i < nr_l ? L.rec[i] : reinterpret_cast<const StageRec*>(sreg + SPILL_OFF_R)[i - nr_l];
  };
  const bool ovf = L.ovf != 0;
  if (!ovf)
    for (int r = tid; r < nr; r += blockDim.x) {
      const int m = rec_at(r).msg;
      if (m != REC_HOLE) atomicAdd(&cntm[m], 1u);
    }
  __syncthreads();
  const uint32_t nh_l16 = ((uint32_t)nh_l + 15u) & ~15u;
  static_assert(TM <= 64, "one wave scans the tile's messages");
  if (tid < 64) {  // wave 0, lane = message: the record base of every message (exclusive scan)
    const int lane = tid;
    const bool live = !ovf && lane < nvalid && L.raise_key[lane] == 0xFFFFFFFFu;
    const uint32_t c = live ? cntm[lane] : 0u;
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane < nvalid) L.mbase[lane] = x - c;
    const uint32_t nrec = __shfl(x, 63);
    // 16-B pieces: full-width copies
    const uint32_t nheap = ovf ? 0u : nh_l16 + (((uint32_t)nh_s + 15u) & ~15u);
    uint32_t got = 0;  // both cursors reserved by one instruction (lanes 0 and 1)
    if (!ovf && lane < 2) got = atomicAdd(&out.cursor_dev[lane], lane == 0 ? nrec : nheap);
    const uint32_t rb = __shfl(got, 0), hb = __shfl(got, 1);
    if (lane == 0) {
      int bad = ovf ? 1 : 0;
      if (!bad) {
        if (rb + nrec > out.rec_cap || hb + nheap > out.heap_cap) {
          bad = 2;
          atomicOr(&out.cursor_dev[2], 1u);
        }
      } else {
        atomicOr(&out.cursor_dev[2], 2u);
      }
      L.tile_bad = bad;
      L.rec_base = rb;
      L.heap_base = hb;
      L.tot_rec = nrec;
    }
  }
  __syncthreads();
  const int bad = L.tile_bad;  // block-uniform
  if (!bad) {
    for (int r = tid; r < nr; r += blockDim.x) {
      const int m = rec_at(r).msg;
      if (m == REC_HOLE || L.raise_key[m] != 0xFFFFFFFFu) continue;
      const uint32_t b = atomicAdd(&fill[m], 1u);
      bidx[L.mbase[m] + b] = (uint16_t)r;
    }
    __syncthreads();
    const int nt = (int)L.tot_rec;
    for (int j = tid; j < nt; j += blockDim.x) {
      const StageRec sr = rec_at(bidx[j]);
      const uint32_t key = ((uint32_t)sr.proto << 16) | sr.rank;
      const uint32_t b0 = L.mbase[sr.msg], b1 = b0 + cntm[sr.msg];
      uint32_t rk = 0;
      for (uint32_t i = b0; i < b1; ++i) {
        const StageRec o = rec_at(bidx[i]);
        rk += (((uint32_t)o.proto << 16) | o.rank) < key ? 1u : 0u;
      }
      sdx_result o;
      o.payload_off = L.heap_base + ((sr.off & HEAP_SPILLED) ? nh_l16 + (sr.off & ~HEAP_SPILLED) : sr.off);
      o.payload_len = sr.len;
      o.proto = sr.proto;
      const bool staged_nib = (sr.bitlen & STAGE_NIB) != 0;
      o.bit_length = staged_nib ? (sr.bitlen & 0xFFFFu) : sr.bitlen;
      o.msg = (uint32_t)msg_of[sr.msg];
      out.rec_dev[L.rec_base + b0 + rk] = o;
      if (wx) {
        uint32_t xr;
        if (staged_nib) {   // classified by the finisher
          const int pl = kind == SDX_KIND_MU ? bv.mu[sr.proto].pre_len : bv.ms[sr.proto].pre_len;
          xr = SDX_XREC_NIB | ((uint32_t)pl << 16) | ((sr.bitlen >> 16) & 0x7FFFu);
        } else if (sr.off & HEAP_SPILLED) {  // two call sites: one pointer per address space (a
          // selected generic pointer here crashed the ROCm 7.2 compiler)
          xr = wire_class(bv, kind, sr.proto, sreg + SPILL_OFF_H + (sr.off & ~HEAP_SPILLED), sr.len);
        } else {
          xr = wire_class(bv, kind, sr.proto, L.heap + sr.off, sr.len);
        }
        if (out.xrec_dev) out.xrec_dev[L.rec_base + b0 + rk] = xr;
        atomicAdd(reinterpret_cast<unsigned long long*>(&wsum[sr.msg]),
                  (unsigned long long)(((uint64_t)sr.len << 32) | wire_bytes_x(xr, sr.len)));
      }
    }
    uint8_t* hd = out.heap_dev + L.heap_base;
    if ((((uintptr_t)hd) & 15u) == 0) {  // 16-B stores (every tile reserves a multiple of 16 B)
      const int n16 = (nh_l + 15) >> 4;
      const uint4* src = reinterpret_cast<const uint4*>(L.heap);
      uint4* dst = reinterpret_cast<uint4*>(hd);
      for (int i = tid; i < n16; i += blockDim.x) dst[i] = src[i];
      const int s16 = (nh_s + 15) >> 4;
      if (s16) {
        const uint4* ssrc = reinterpret_cast<const uint4*>(sreg + SPILL_OFF_H);
        uint4* sdst = reinterpret_cast<uint4*>(hd + nh_l16);
        for (int i = tid; i < s16; i += blockDim.x) sdst[i] = ssrc[i];
      }
    } else {
      for (int i = tid; i < nh_l; i += blockDim.x) hd[i] = L.heap[i];
      for (int i = tid; i < nh_s; i += blockDim.x) hd[nh_l16 + i] = sreg[SPILL_OFF_H + i];
    }
  }
  if (wx) __syncthreads();  // wsum complete (block-uniform)
  for (int m = tid; m < nvalid; m += blockDim.x) {
    sdx_desc d;
    d.rec_begin = L.rec_base + L.mbase[m];
    const uint32_t rk = L.raise_key[m];
    if (rk != 0xFFFFFFFFu) {
      d.status = SDX_ST_RAISED;
      d.raise_kind = (uint8_t)(rk & 0xFF);
      d.n_rec = 0;
    } else if (bad) {
      d.status = bad == 2 ? SDX_ST_OVF_OUT : SDX_ST_OVF_TILE;
      d.raise_kind = 0;
      d.n_rec = 0;
    } else {
      d.status = SDX_ST_OK;
      d.raise_kind = 0;
      d.n_rec = (uint16_t)cntm[m];
    }
    out.desc_dev[msg_of[m]] = d;
    if (wx) out.wire_dev[msg_of[m]] = d.status == SDX_ST_OK ? wsum[m] : 0ull;
  }
}

// ---------------------------------------------------------------------------------------------
// MU / MS tile kernel
// ---------------------------------------------------------------------------------------------
// the lane-decode MU variant runs 8 waves per tile; (512, 2) asks for 2 such tiles per CU,
// i.e. 4 waves/SIMD (<= 128 VGPRs)
template <int KIND, int NW>
constexpr int pulses_threads() { return NW <= 4 ? 64 * LANE_WAVES : 256; }
template <int KIND, int NW>
constexpr int pulses_min_blocks() { return NW <= 4 ? 16 / LANE_WAVES : 1; }

// MR = 1: the short variant reads its header fields from the message records (b.mrec_dev); a
// separate instantiation, so the default one carries no trace of that path.
// SPLIT (MS, one launch per length class over the same tiles): > 0 = this launch takes the tiles
// whose longest message has more than 64 * (SPLIT - 1) and at most 64 * NW pulses; a tile that is not
// its launch's returns before it touches anything (a block-uniform test on the tile's lengths)
template <int KIND, int NW, int TM>
using PulsesLds = TileLds<NW, TM, (KIND == SDX_KIND_MU && NW <= 4) ? 1 : ((KIND == SDX_KIND_MS && NW <= 4) ? 2 : 0)>;

// one tile (TM messages, blk = the tile's index in the launch) of a k_pulses launch; the tile's LDS
// and message list come from the calling kernel (k_pulses, or k_step's union)
template <int KIND, int NW, int TM, int MR, int SPLIT>
SDX_DEV void pulses_tile(const void* __restrict__ bank, const sdx_pulse_batch& b, const sdx_out& out, const int blk,
                         PulsesLds<KIND, NW, TM>& L, int* msg_of) {
  constexpr bool LANE_MU = KIND == SDX_KIND_MU && NW <= 4;
  constexpr bool LANE_MS = KIND == SDX_KIND_MS && NW <= 4;
  using T = PulsesLds<KIND, NW, TM>;
  const BankView bv = bank_view(bank);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int tile0 = blk * TM;
  const int nvalid = (ntot - tile0 < TM) ? ntot - tile0 : TM;
#ifdef SDX_WGTIME
  if (tid == 0 && blk < 65536) g_wgt[2 * blk] = __builtin_amdgcn_s_memrealtime();
#endif
  if constexpr (SPLIT != 0) {
    int len = 0;
    if (tid < nvalid) {
      const int msg = b.sel_dev ? b.sel_dev[tile0 + tid] : tile0 + tid;
      const int64_t o = b.offsets_dev[msg];
      len = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - o);
    }
    const bool above = __syncthreads_or(len > 64 * NW) != 0;           // another launch's (wider) tile
    const bool below = SPLIT == 1 || __syncthreads_or(len > 64 * (SPLIT - 1)) != 0;
    if (above || !below) return;
  }
  if (tid < TM) {
    msg_of[tid] = (tid < nvalid) ? (b.sel_dev ? b.sel_dev[tile0 + tid] : tile0 + tid) : 0;
    L.raise_key[tid] = 0xFFFFFFFFu;
    L.cnt[tid] = 0;
  }
  if (tid == 0) {
    L.next_p = 0;
    L.nmatch = 0;
    L.pool_ctr = 0;
    L.spill_base = SPILL_NONE;
    L.sp_rec = 0;
    L.sp_heap = 0;
    L.ovf = 0;
    L.nsurv = 0;
  }
  if constexpr (LANE_MU) {  // MU decode descriptors + modulematch tables -> LDS (16-B pieces)
    const int ndesc = (int)bv.hdr->n_mu < SDX_MUDESC_LDS ? (int)bv.hdr->n_mu : SDX_MUDESC_LDS;
    const int n16 = (ndesc * (int)sizeof(sdx_mu_desc) + 15) >> 4;
    const uint4* src = reinterpret_cast<const uint4*>(bv.mudesc);
    uint4* dst = reinterpret_cast<uint4*>(L.desc);
    for (int i = tid; i < n16; i += blockDim.x) dst[i] = src[i];
    if (tid == 0) L.mm_states = (int)bv.hdr->mm_states;
  }
  if constexpr (LANE_MS) {
    const int nd = (int)bv.hdr->n_ms < MS_DESC_LDS ? (int)bv.hdr->n_ms : MS_DESC_LDS;
    for (int i = tid; i < nd; i += blockDim.x) L.msdesc[i] = ms_desc(bv.ms + i);
  }
#ifdef SDX_PROF
  if (lane < 28) L.prof[wave][lane] = 0;
#endif
  __syncthreads();
  PROF_T(t_kernel);
  PROF_T(t_stage);
  // ---- stage: per-id position bitmaps (coalesced 64-character rows, 10 ballots each)
  constexpr int NWAVE = pulses_threads<KIND, NW>() / 64;
  // short variants: a wave's messages are fetched up front -- lane k loads message k's offset and
  // length, then every message's characters are loaded into registers -- so the global-load
  // latencies of the wave's messages overlap instead of adding up message after message
  constexpr int MPW = NW <= 4 ? (TM + NWAVE - 1) / NWAVE : 1;
  // short variants: the tile's pattern tables, one thread per (message, pattern) with consecutive
  // addresses, into the result pool's heap (unused until the finish phase): every wave then reads
  // its lanes' patterns from LDS instead of each of the NWAVE waves loading them strided from HBM.
  //   MU: x = 10|P| (integral P, |P| < 2^26) for the integer normalisation, flags (bit0 sign, bit1 fp64 path)
  //   MS: k of round(P / abs(P[CP]), 1) (message_synced.py:64-72) and the clock abs(P[CP])
  static_assert(T::PHEAP >= TM * SDX_MAXPAT * 6 + TM * 16, "pattern staging fits the pool heap");
  uint32_t* st_x = reinterpret_cast<uint32_t*>(L.heap);                    // [TM][10]
  uint8_t* st_f = L.heap + TM * SDX_MAXPAT * 4;                            // [TM][10]
  uint8_t* st_id = st_f + TM * SDX_MAXPAT;                                 // [TM][10]
  double* st_clk = reinterpret_cast<double*>(st_id + TM * SDX_MAXPAT);     // [TM] (MS)
  uint8_t* st_np = reinterpret_cast<uint8_t*>(st_clk + TM);                // [TM]
  int64_t pf_off = 0;
  int pf_n = 0;
  // SWAR staging (short variants): 16 characters per lane, 4 messages per pass over the wave
  constexpr int LPM = NW <= 4 ? 4 * NW : 16;        // lanes per message (16 characters each)
  constexpr int SMSG = 64 / LPM;                    // messages per pass
  constexpr int SPASS = (MPW + SMSG - 1) / SMSG;   // passes per wave
  static_assert(NW > 4 || NW == 4 || NW == 2, "SWAR staging: 128- or 256-character rows");
  uint32_t sx[NW <= 4 ? SPASS : 1][5];
  if constexpr (NW <= 4) {
    // every header load of the tile is issued before any of them is used: the data offsets of the
    // wave's messages, and per (message, pattern) thread npat, P, the id and (MS) the message's
    // CP slot with all its values (five 16-B loads; the clock is selected in registers) -- two
    // levels of dependent global loads (message index -> fields -> data) instead of five
    // with message records (b.mrec_dev, written by the grouping in message order) every header
    // field of a message comes from its one 128-byte line instead of a scattered sector per field
    const sdx_msg_rec* __restrict__ mrec = MR ? b.mrec_dev : nullptr;
    if (lane < MPW && wave + lane * NWAVE < nvalid) {
      const int msg = msg_of[wave + lane * NWAVE];
      if (mrec) {
        const int4 h = *reinterpret_cast<const int4*>(mrec + msg);
        pf_off = (int64_t)(((uint64_t)(uint32_t)h.y << 32) | (uint32_t)h.x);
        pf_n = h.z;
      } else {
        pf_off = b.offsets_dev[msg];
        pf_n = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - pf_off);
      }
      if (pf_n > 64 * NW) pf_n = 64 * NW;
    }
    constexpr int NTH = pulses_threads<KIND, NW>();
    constexpr int NIT = (TM * SDX_MAXPAT + NTH - 1) / NTH;
    int r_np[NIT], r_cp[NIT];
    double r_v[NIT];
    uint8_t r_id[NIT];
    double2 r_all[NIT][KIND == SDX_KIND_MS ? SDX_MAXPAT / 2 : 1];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + it * NTH;
      const int m = i / SDX_MAXPAT, k = i - m * SDX_MAXPAT;
      const bool ok = i < TM * SDX_MAXPAT && m < nvalid;
      const int msg = ok ? msg_of[m] : 0;
      if (mrec) {
        const sdx_msg_rec* r = mrec + msg;
        r_np[it] = ok ? (int)r->npat : 0;
        r_v[it] = ok ? r->pat_val[k] : 0.0;
        r_id[it] = ok ? r->pat_id[k] : (uint8_t)'0';
      } else {
        r_np[it] = ok ? (int)b.npat_dev[msg] : 0;
        r_v[it] = ok ? b.pat_val_dev[msg * SDX_MAXPAT + k] : 0.0;  // n x 10 values: always in bounds
        r_id[it] = ok ? b.pat_id_dev[msg * SDX_MAXPAT + k] : (uint8_t)'0';
      }
      r_cp[it] = -1;
      if constexpr (KIND == SDX_KIND_MS) {
        r_cp[it] = ok ? (int)(mrec ? mrec[msg].cp_slot : b.cp_slot_dev[msg]) : -1;
        const double2* row = mrec ? reinterpret_cast<const double2*>(mrec[msg].pat_val)
                                  : reinterpret_cast<const double2*>(b.pat_val_dev + msg * SDX_MAXPAT);
#pragma unroll
        for (int h = 0; h < SDX_MAXPAT / 2; ++h) r_all[it][h] = ok ? row[h] : make_double2(0.0, 0.0);
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = tid + it * NTH;
      const int m = i / SDX_MAXPAT, k = i - m * SDX_MAXPAT;
      if (!(i < TM * SDX_MAXPAT && m < nvalid)) continue;
      const int np = r_np[it] > SDX_MAXPAT ? SDX_MAXPAT : r_np[it];
      if (k == 0) st_np[m] = (uint8_t)np;
      if (k >= np) continue;
      const double v = r_v[it];
      st_id[i] = (uint8_t)((r_id[it] - '0') & 15);
      if constexpr (KIND == SDX_KIND_MU) {
        const double av = fabs(v);
        const bool fast = av < 67108864.0 && av == floor(av);  // 2^26; NaN fails
        st_x[i] = fast ? (uint32_t)av * 10u : 0u;
        st_f[i] = (uint8_t)((signbit(v) ? 1 : 0) | (fast ? 0 : 2));
      } else {
        const int cp = r_cp[it];
        double pc = 0.0;
#pragma unroll
        for (int h = 0; h < SDX_MAXPAT / 2; ++h) {
          if (cp == 2 * h) pc = r_all[it][h].x;
          if (cp == 2 * h + 1) pc = r_all[it][h].y;
        }
        const double clk = (cp >= 0 && cp < np) ? fabs(pc) : 0.0;
        if (k == 0) st_clk[m] = clk;
        st_x[i] = (uint32_t)(clk != 0.0 ? py_round1_k(v / clk) : SDX_K_NONE);
      }
    }
    PROF_ADD(17, t_stage);
    // 16 characters per lane: lane group g = lane / 16 holds tile message 4 * pass + g, lane j = lane % 16
    // its characters [16 j, 16 j + 16) as five aligned dwords (realigned below; a dword that holds a
    // byte of the message cannot cross a page, so the loads past the message end stay in bounds)
#pragma unroll
    for (int ps = 0; ps < SPASS; ++ps) {
      const int k = ps * SMSG + lane / LPM;
      const int lo = __shfl((int)(uint32_t)pf_off, k), hi = __shfl((int)(uint32_t)((uint64_t)pf_off >> 32), k);
      const int64_t off = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
      const int n = __shfl(pf_n, k);
      const int64_t base = off + 16 * (lane % LPM);
      const int64_t a = base & ~(int64_t)3;
      const bool on = wave + k * NWAVE < nvalid;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(b.data_dev + a);
#pragma unroll
      for (int i = 0; i < 5; ++i) sx[ps][i] = (on && a + 4 * i < off + n) ? src[i] : 0xFFFFFFFFu;
    }
  }
  PROF_T(t_bm);
  if constexpr (NW <= 4) {
  // per pass: the lane's 16 characters -> 10 id masks of 16 bits (SWAR on 4 characters per dword),
  // written as 16-bit pieces of the per-id bitmaps; non-digit characters per message by ballot
  uint32_t ndmsg = 0;  // bit k: tile message k of the wave holds a non-digit character
#pragma unroll
  for (int ps = 0; ps < SPASS; ++ps) {
    const int k = ps * SMSG + lane / LPM, j = lane % LPM;
    const int mi = wave + k * NWAVE;
    const int n = __shfl(pf_n, k);
    const int lo = __shfl((int)(uint32_t)pf_off, k);
    const uint32_t r = (uint32_t)lo & 3u;  // realignment of the message's rows
    uint32_t V = 0, P0 = 0, P1 = 0, P2 = 0, P3 = 0, FE = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t c = __builtin_amdgcn_alignbyte(sx[ps][i + 1], sx[ps][i], r);  // bytes r.. of the pair
      const int rem = n - (16 * j + 4 * i);  // characters of this dword inside the message
      c = rem >= 4 ? c : (rem <= 0 ? 0xFFFFFFFFu : (c | (0xFFFFFFFFu << (8 * rem))));
      const uint32_t t = c ^ 0x30303030u;        // digits -> 0x00..0x09
      const uint32_t lo4 = t & 0x0F0F0F0Fu;
      const uint32_t bad = (t & 0xF0F0F0F0u) | ((lo4 + 0x06060606u) & 0x10101010u);  // byte != 0 <=> not a digit
      const uint32_t nz = ((bad & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | bad;               // bit 7: byte != 0
      const uint32_t dg = (~nz >> 7) & 0x01010101u;                                // byte bit 0: digit
      V |= ((dg * 0x01020408u) >> 24) << (4 * i);
      P0 |= (((lo4 & 0x01010101u) * 0x01020408u) >> 24) << (4 * i);
      P1 |= (((lo4 & 0x02020202u) * 0x00810204u) >> 24) << (4 * i);
      P2 |= (((lo4 & 0x04040404u) * 0x00408102u) >> 24) << (4 * i);
      P3 |= (((lo4 & 0x08080808u) * 0x00204081u) >> 24) << (4 * i);
      if (__builtin_expect(bad != 0 && rem > 0, 0)) {  // 0xFE counts as isdigit() (packing.py), not as an id
        const uint32_t fe = c ^ 0xFEFEFEFEu;
        const uint32_t fz = ~(((fe & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | fe) & 0x80808080u;
        FE |= ((((fz >> 7) & 0x01010101u) * 0x01020408u) >> 24) << (4 * i);
      }
    }
    const uint32_t posm = n - 16 * j >= 16 ? 0xFFFFu : (n - 16 * j <= 0 ? 0u : (1u << (n - 16 * j)) - 1u);
    const bool nondigit = (posm & ~V & ~FE) != 0;
    const uint64_t ndb = ballot(nondigit);
#pragma unroll
    for (int g = 0; g < SMSG; ++g)
      if ((ndb >> (LPM * g)) & ((1ull << LPM) - 1)) ndmsg |= 1u << (ps * SMSG + g);
    if (mi < nvalid) {
      const uint32_t N0 = ~P0, N1 = ~P1, N2 = ~P2, N3 = ~P3;
      uint16_t* row = reinterpret_cast<uint16_t*>(&L.bm[mi * T::MSTRIDE + (j >> 2)]) + (j & 3);
#pragma unroll
      for (int id = 0; id < 10; ++id) {
        const uint32_t m = V & ((id & 1) ? P0 : N0) & ((id & 2) ? P1 : N1) & ((id & 4) ? P2 : N2) &
                           ((id & 8) ? P3 : N3);
        row[id * T::WS * 4] = (uint16_t)m;
      }
    }
  }
  wave_sync();
  PROF_ADD(18, t_bm);
  PROF_T(t_pairs);
#pragma unroll
  for (int k = 0; k < MPW; ++k) {
    const int mi = wave + k * NWAVE;
    if (mi >= nvalid) break;
    const int n = __shfl(pf_n, k);
    const int nwu = (n + 63) >> 6;  // words holding pulses (wave-uniform); the rest are empty
    const uint64_t nd = (ndmsg >> k) & 1u;
    if constexpr (NW <= 4) {  // pair presence: lane = id pair (a, b), a = q / 10, b = q % 10
      wave_sync();
      uint64_t pr[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = lane + 64 * h;
        uint64_t acc = 0;
        if (q < 100) {
          const uint64_t* A = &L.bm[mi * T::MSTRIDE + (q / 10) * T::WS];
          const uint64_t* B = &L.bm[mi * T::MSTRIDE + (q % 10) * T::WS];
#pragma unroll
          for (int w = 0; w < NW; ++w)
            if (KIND != SDX_KIND_MS || w < nwu) acc |= A[w] & ((B[w] >> 1) | (w + 1 < NW ? B[w + 1] << 63 : 0ull));
        }
        pr[h] = ballot(acc != 0);
      }
      if (lane == 0) {
        L.pairs[mi][0] = pr[0];
        L.pairs[mi][1] = pr[1];
      }
    }
    if (lane == 0) {
      L.nlen[mi] = n;
      L.digit_ok[mi] = (nd == 0 && n > 0) ? 1u : 0u;
    }
  }
  PROF_ADD(19, t_pairs);
  }
  if constexpr (NW > 4) {  // long variants: one message per wave
    for (int mi = wave; mi < nvalid; mi += NWAVE) {
      const int msg = msg_of[mi];
      const int64_t off = b.offsets_dev[msg];
      int n = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
      if (n > 64 * NW) n = 64 * NW;
      bool nondigit = false;
      for (int w = 0; w < NW; ++w) {
        const int pos = w * 64 + lane;
        const uint8_t c = pos < n ? b.data_dev[off + pos] : (uint8_t)0xFF;
        nondigit |= pos < n && !((c >= '0' && c <= '9') || c == 0xFE);
        uint64_t mine = 0;
#pragma unroll
        for (int id = 0; id < 10; ++id) {
          const uint64_t bb = ballot(c == (uint8_t)('0' + id));
          if (lane == id) mine = bb;
        }
        if (lane < 10) L.bm[mi * T::MSTRIDE + lane * T::WS + w] = mine;
      }
      const uint64_t nd = ballot(nondigit);
      if (lane == 0) {
        L.nlen[mi] = n;
        L.digit_ok[mi] = (nd == 0 && n > 0) ? 1u : 0u;
      }
    }
  }
  __syncthreads();
  PROF_ADD(0, t_stage);
  // ---- per-lane message state (lane = message of the tile)
  const int mi = lane;
  const bool mvalid = mi < nvalid;
  int npat = 0, n = 0;
  uint64_t ids = 0;
  double val[SDX_MAXPAT];
  int kq[SDX_MAXPAT];  // normalised pattern values round(x / clock, 1) == kq / 10 (SDX_K_NONE: absent)
#pragma unroll
  for (int k = 0; k < SDX_MAXPAT; ++k) {
    val[k] = 0.0;
    kq[k] = SDX_K_NONE;
  }
  bool lane_ok = false;
  // MU (lane variant): the integer form of every pattern value for the per-clock normalisation,
  // x = 10 * |P| when P is integral and |P| < 2^26 (bit k of slowm otherwise: fp64 path), sign in negm
  uint32_t xk[SDX_MAXPAT];
  uint32_t negm = 0, slowm = 0;
#pragma unroll
  for (int k = 0; k < SDX_MAXPAT; ++k) xk[k] = 0;
  if (mvalid) {
    const int msg = msg_of[mi];
    if constexpr (NW <= 4) {  // the staged pattern tables
      npat = st_np[mi];
#pragma unroll
      for (int k = 0; k < SDX_MAXPAT; ++k) {
        if (k < npat) {
          const int i = mi * SDX_MAXPAT + k;
          ids |= (uint64_t)st_id[i] << (4 * k);
          if constexpr (LANE_MU) {
            xk[k] = st_x[i];
            const uint32_t f = st_f[i];
            negm |= (f & 1u) << k;
            slowm |= ((f >> 1) & 1u) << k;
          } else {
            kq[k] = (int)st_x[i];  // MS: k staged (normalised once, by the message's own clock)
          }
        }
      }
    } else {
      npat = b.npat_dev[msg];
      if (npat > SDX_MAXPAT) npat = SDX_MAXPAT;
#pragma unroll
      for (int k = 0; k < SDX_MAXPAT; ++k) {
        if (k < npat) {
          ids |= (uint64_t)((b.pat_id_dev[msg * SDX_MAXPAT + k] - '0') & 15) << (4 * k);
          val[k] = b.pat_val_dev[msg * SDX_MAXPAT + k];
        }
      }
    }
    n = L.nlen[mi];
    lane_ok = n > 0;  // empty D -> [] (message_unsynced.py:22-25 / message_synced.py:23-25)
  }
  PairRef PR{0, 0};
  if constexpr (NW <= 4) {
    if (mvalid) {
      PR.P0 = L.pairs[mi][0];
      PR.P1 = L.pairs[mi][1];
    }
  }
  const uint64_t* bmine = &L.bm[(mvalid ? mi : 0) * T::MSTRIDE];
  const int nw = (n + 63) >> 6;
  double clock = 0.0;
  if (KIND == SDX_KIND_MS && mvalid) {
    // gates (message_synced.py:21-66): data.isdigit(), CP/SP/R string checks, CP in patterns, clock != 0
    const int msg = msg_of[mi];
    const bool use_rec = MR && NW <= 4;
    const int cp = use_rec ? b.mrec_dev[msg].cp_slot : b.cp_slot_dev[msg];
    const bool ok_ms = use_rec ? b.mrec_dev[msg].ms_ok : b.ms_ok_dev[msg];
    lane_ok = lane_ok && L.digit_ok[mi] && ok_ms && cp >= 0 && cp < npat;
    if constexpr (NW <= 4) {  // clock and k were staged (st_clk / st_x)
      clock = st_clk[mi];
      lane_ok = lane_ok && clock != 0.0;
      if (!lane_ok) {
#pragma unroll
        for (int k = 0; k < SDX_MAXPAT; ++k) kq[k] = SDX_K_NONE;
      }
    } else {
#pragma unroll
      for (int k = 0; k < SDX_MAXPAT; ++k)
        if (k == cp) clock = fabs(val[k]);
      lane_ok = lane_ok && clock != 0.0;
      if (lane_ok) {
#pragma unroll
        for (int k = 0; k < SDX_MAXPAT; ++k)
          if (k < npat) kq[k] = py_round1_k(val[k] / clock);
      }
    }
  }
  // pattern_exists: lane variant on a SpecV (compact MU filter record or full patspec), long
  // variant on the full patspec
  auto PEXV = [&](const SpecV& sv, const sdx_patspec* sp, int minpos, bool need_pos) -> PexRes {
    if constexpr (NW <= 4) return pexists_lane<NW>(sv, kq, ids, npat, bmine, minpos, bv.rank, PR, need_pos);
    else return pattern_exists(sp, kq, ids, npat, bmine, T::WS, nw, minpos);
  };
  // ---- protocol loop: waves take protocols one at a time, in the bank's processing order
  // (MU: sorted by clock), from a tile counter -- results are ordered at the flush, so the
  // processing order is free and dynamic assignment balances the waves
  const int nproto = KIND == SDX_KIND_MU ? (int)bv.hdr->n_mu : (int)bv.hdr->n_ms;
  const uint16_t* order = bv.order + (KIND == SDX_KIND_MU ? 0 : (int)bv.hdr->n_mu);
  double last_clock = __builtin_nan("");  // NaN != anything: the first protocol normalises
  MuItem* Q = nullptr;
  int q_head = 0, q_tail = 0;
  if constexpr (LANE_MU) Q = L.u.q[wave];
  auto drain = [&](int head, int cnt) {
    wave_sync();
    if constexpr (KIND == SDX_KIND_MU && NW <= 4) {
      if (lane < cnt) {
        const MuItem it = Q[(head + lane) & (QCAP - 1)];
        const int qm = it.mi, qp = it.p;
        const uint32_t rk = L.raise_key[qm];
        if (rk == 0xFFFFFFFFu || (rk >> 8) > (uint32_t)qp) {
          sdx_mu_desc d;
          if (qp < SDX_MUDESC_LDS) d = L.desc[qp];
          else d = bv.mudesc[qp];
          PROF_CNTL(21);
          decode_mu_lane<NW>(L, out, wave, bv, bv.mu + qp, d, qp, qm, &L.bm[qm * T::MSTRIDE], L.nlen[qm], it.idx,
                             ((uint64_t)it.st_hi << 32) | it.st_lo, it.u0, it.u1, it.u2, it.fmask);
        }
      }
    }
    wave_sync();
  };
  // MU: a wave takes a whole clock group (one normalisation per group); MS: one protocol
  const int ngrab = KIND == SDX_KIND_MU ? (int)bv.hdr->n_mu_groups : nproto;
  const uint16_t* gstart = bv.order + bv.hdr->n_mu + bv.hdr->n_ms;
  int cur = 0, cend = 0;
#ifdef SDX_PROF
  int g_cur = -1;
  unsigned long long g_t0 = 0;
#endif
  while (true) {
    if (cur == cend) {
      int g = 0;
      if (lane == 0) g = atomicAdd(&L.next_p, 1);
      g = __builtin_amdgcn_readfirstlane(g);
#ifdef SDX_PROF
      if (g_cur >= 0 && g_cur < 128 && lane == 0) {
        atomicAdd(&g_gprof[0][g_cur], __builtin_amdgcn_s_memtime() - g_t0);
        atomicAdd(&g_gprof[1][g_cur], 1ull);
      }
      g_cur = g;
      g_t0 = __builtin_amdgcn_s_memtime();
#endif
      if (g >= ngrab) break;
      if (KIND == SDX_KIND_MU) {
        cur = cld(&gstart[g]);
        cend = cld(&gstart[g + 1]);
      } else {
        cur = g;
        cend = g + 1;
      }
    }
    const int p = cld(&order[cur]);
    ++cur;
    if constexpr (KIND == SDX_KIND_MU) {
      const sdx_mu_proto* rec = uniform_ptr(bv.mu + p);
      const sdx_mu_filt* fr = uniform_ptr(bv.mufilt + p);  // the filter's state: two 64-byte lines
      const uint32_t ff = cld(&fr->flags);
      if ((ff & 2u) || !(ff & 4u)) continue;  // never / not active
      const bool full = (ff & 8u) != 0;
      // (a raise of this message in an earlier protocol: the flush drops all its results anyway, so
      // the test only saves work; SDX_NO_RAISE_CHECK A/B)
      bool alive = lane_ok && (SDX_NO_RAISE_CHECK || (L.raise_key[mi] >> 8) > (uint32_t)p || L.raise_key[mi] == 0xFFFFFFFFu);
      int idx = 0;
      uint64_t st_tgt = 0, ut0 = 0, ut1 = 0, ut2 = 0;
      int fmask = 0;
      PROF_T(t_norm);
      const double pclk = cld(&fr->clock);
      if (pclk != last_clock) {  // wave-uniform: consecutive protocols often share a clock
        last_clock = pclk;
        if constexpr (LANE_MU) {
          // round(P / clock, 1) == k / 10 (message_unsynced.py:64): for integral P and an integral
          // clock, k = round-half-even(10|P| / |clock|) with the signs applied -- exact, because
          // fl(P / clock) differs from the rational by < 2^-23 while a non-tie is >= 1 / (2 |clock|)
          // from a rounding boundary.  An exact rational tie |P| / |clock| == (2q + 1) / 20 rounds
          // like fl((2q + 1) / 20): both are the correctly rounded quotient of the same rational,
          // so py_round1_k of it needs no pattern value (it used to reload P from HBM: MU 1.119-1.128
          // -> 1.111-1.114 ms, profiles/r04/ab_tie.log).  Non-integral P and clocks outside the
          // divider's range use py_round1_k on fl(P / clock).
          const uint32_t csh = cld(&fr->clk_sh);
          const uint32_t cc = cld(&fr->clk_c), cm = cld(&fr->clk_m), sh = csh & 0xFFu;
          const bool ivalid = (csh & 0x100u) != 0, cneg = (csh & 0x200u) != 0;
#pragma unroll
          for (int k = 0; k < SDX_MAXPAT; ++k) {
            if (k < npat) {
              const bool slow = !ivalid || ((slowm >> k) & 1u);
              const bool negk = ((negm >> k) & 1u) != 0;
              int kk = 0;
              if (!slow) {
                const uint32_t x = xk[k];
                const uint32_t q = (uint32_t)(((uint64_t)x * cm) >> sh);
                const int d2 = 2 * (int)(x - q * cc) - (int)cc;
                kk = (int)q + (d2 > 0 ? 1 : 0);
                if (d2 == 0) kk = py_round1_k((double)(2 * q + 1) / 20.0);  // exact rational tie
                if (negk != cneg) kk = -kk;
              }
              if (slow) kk = py_round1_k(b.pat_val_dev[msg_of[mi] * SDX_MAXPAT + k] / pclk);
              kq[k] = kk;
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < SDX_MAXPAT; ++k)
            if (k < npat) kq[k] = py_round1_k(val[k] / pclk);
        }
      }
      PROF_ADD(1, t_norm);
      auto SV = [&](int key, const sdx_patspec* sp) -> SpecV {
        if constexpr (NW <= 4) {
          if (!full) return spec_compact(&fr->spec[key], key == 0 ? cld(&fr->start_upk) : (uint64_t)cld(&fr->spec[key].upk));
          return spec_full(sp);
        } else {
          return SpecV{};
        }
      };
      PROF_T(t_st);
      if (alive) {
        if (ff & 1u) {
          const PexRes r = PEXV(SV(0, &rec->start), &rec->start, 0, true);
          alive = r.found;
          idx = r.pos;
          st_tgt = r.tgt;
        }
      }
      PROF_ADD(2, t_st);
      PROF_T(t_ozf);
      auto klen = [&](int key) -> int { return (int)((cld(&fr->spec[key].rk2_len_nu) >> 16) & 0xFF); };
      if (alive && klen(1)) {
        const PexRes r = PEXV(SV(1, &rec->one), &rec->one, idx, false);
        if (r.found) { ut0 = r.tgt; fmask |= 1; } else alive = false;
      }
      if (alive && klen(2)) {
        const PexRes r = PEXV(SV(2, &rec->zero), &rec->zero, idx, false);
        if (r.found) { ut1 = r.tgt; fmask |= 2; } else alive = false;
      }
      if (alive && klen(3)) {
        const PexRes r = PEXV(SV(3, &rec->flt), &rec->flt, idx, false);
        if (r.found) { ut2 = r.tgt; fmask |= 4; }
      }
      alive = alive && fmask != 0;
      PROF_ADD(3, t_ozf);
      PROF_T(t_dec);
      if constexpr (NW <= 4) {
        // queue the survivors; drain 64 at a time with lane = (message, protocol) pair
        const uint64_t pass = ballot(alive);
        if (pass) {
          if (alive) {
            MuItem it;
            it.st_lo = (uint32_t)st_tgt;
            it.st_hi = (uint32_t)(st_tgt >> 32);
            it.u0 = (uint16_t)ut0;
            it.u1 = (uint16_t)ut1;
            it.u2 = (uint16_t)ut2;
            it.idx = (uint16_t)idx;
            it.p = (uint16_t)p;
            it.mi = (uint8_t)mi;
            it.fmask = (uint8_t)fmask;
            Q[(q_tail + lanes_below(pass)) & (QCAP - 1)] = it;
          }
          q_tail += popc64(pass);
          if (q_tail - q_head >= WAVE) {
            drain(q_head, WAVE);
            q_head += WAVE;
          }
        }
      } else {
        uint64_t surv = ballot(alive);
        while (surv) {
          const int sl = ffs64(surv);
          surv &= surv - 1;
          decode_mu(L, wave, bv, rec, p, sl, bcast_i(idx, sl), bcast_u64(st_tgt, sl), bcast_u64(ut0, sl),
                    bcast_u64(ut1, sl), bcast_u64(ut2, sl), bcast_i(fmask, sl));
        }
      }
      PROF_ADD(12, t_dec);
    } else {
      const sdx_ms_proto* rec = uniform_ptr(bv.ms + p);
      const sdx_ms_filt* fr = uniform_ptr(bv.msfilt + p);  // the filter's state: two 64-byte lines
      const uint32_t ff = cld(&fr->flags);
      if (ff & 2u) continue;  // never
      const bool full = (ff & 8u) != 0;
      // the lane variant decodes after the loop, so no message of the tile has raised yet here
      bool alive = lane_ok && ((LANE_MS && SDX_NO_RAISE_CHECK) || (L.raise_key[mi] >> 8) > (uint32_t)p ||
                               L.raise_key[mi] == 0xFFFFFFFFu);
      const double pclk = cld(&fr->pclock);
      if (alive && pclk > 0.0)  // clock tolerance gate (:83-88)
        alive = !(fabs(pclk - clock) > clock * 0.3);
      int start = 0;
      uint64_t kt0 = 0, kt1 = 0, kt2 = 0, kt3 = 0;
      int fmask = 0;
      auto SV = [&](int key) -> SpecV {
        if constexpr (NW <= 4) {
          if (!full) return spec_compact(&fr->spec[key], key == 0 ? cld(&fr->sync_upk) : (uint64_t)cld(&fr->spec[key].upk));
          return spec_full(&rec->key[key]);
        } else {
          return SpecV{};
        }
      };
      auto klen = [&](int key) -> int { return (int)((cld(&fr->spec[key].rk2_len_nu) >> 16) & 0xFF); };
      if (alive && klen(0)) {  // sync (:140-158)
        const PexRes r = PEXV(SV(0), &rec->key[0], 0, true);
        if (r.found) {
          kt0 = r.tgt;
          fmask |= 1;
          start = r.pos + klen(0);
          const int width = cld(&fr->width);
          const double avail = width > 0 ? (double)(n - start) / (double)width : 0.0;
          if ((double)cld(&fr->lmin_sync) > avail) alive = false;
        } else alive = false;
      }
      if (alive && klen(1)) {
        const PexRes r = PEXV(SV(1), &rec->key[1], 0, false);
        if (r.found) { kt1 = r.tgt; fmask |= 2; } else alive = false;
      }
      if (alive && klen(2)) {
        const PexRes r = PEXV(SV(2), &rec->key[2], 0, false);
        if (r.found) { kt2 = r.tgt; fmask |= 4; } else alive = false;
      }
      if (alive && klen(3)) {
        const PexRes r = PEXV(SV(3), &rec->key[3], 0, false);
        if (r.found) { kt3 = r.tgt; fmask |= 8; }
      }
      alive = alive && fmask != 0;
      if constexpr (LANE_MS) {  // append the survivors to the tile list (decoded after the loop)
        const uint64_t pass = ballot(alive);
        if (pass) {
          int base = 0;
          if (lane == 0) base = atomicAdd(&L.nsurv, popc64(pass));
          base = __builtin_amdgcn_readfirstlane(base);
          const int slot = base + lanes_below(pass);
          if (alive && slot < MS_SURV_CAP) {
            MsItem it;
            it.k0_lo = (uint32_t)kt0;
            it.k0_hi = (uint32_t)(kt0 >> 32);
            it.k1 = (uint16_t)kt1;
            it.k2 = (uint16_t)kt2;
            it.k3 = (uint16_t)kt3;
            it.start = (uint16_t)start;
            it.p = (uint16_t)p;
            it.mi = (uint8_t)mi;
            it.fmask = (uint8_t)fmask;
            L.slist[slot] = it;
          }
          if (base + popc64(pass) > MS_SURV_CAP && lane == 0) L.ovf = 1;  // tile re-run (long variant)
        }
      } else {
        uint64_t surv = ballot(alive);
        while (surv) {
          const int sl = ffs64(surv);
          surv &= surv - 1;
          decode_ms(L, wave, bv, rec, p, sl, bcast_i(start, sl), bcast_u64(kt0, sl), bcast_u64(kt1, sl),
                    bcast_u64(kt2, sl), bcast_u64(kt3, sl), bcast_i(fmask, sl));
        }
      }
    }
  }
  if constexpr (LANE_MU) {
    PROF_T(t_dec);
    while (q_head < q_tail) {
      const int c = (q_tail - q_head < WAVE) ? q_tail - q_head : WAVE;
      drain(q_head, c);
      q_head += c;
    }
    PROF_ADD(12, t_dec);
  }
  PROF_T(t_bar);
  __syncthreads();
  PROF_ADD(14, t_bar);
  if constexpr (LANE_MS) {  // decode every survivor of the tile: lane = (message, protocol)
    PROF_T(t_dec);
    const int ns = L.nsurv < MS_SURV_CAP ? L.nsurv : MS_SURV_CAP;
    if (!L.ovf) {
      // survivors packed into the first waves (dealing them round-robin over all 8 measured
      // 0.73 vs 0.645 ms: more waves on the same divergent decode path)
      for (int i = tid; i < ns; i += blockDim.x) {
        const MsItem it = L.slist[i];
        const int qm = it.mi, qp = it.p;
        const uint32_t rk = L.raise_key[qm];
        if (rk == 0xFFFFFFFFu || (rk >> 8) > (uint32_t)qp)
          decode_ms_lane<NW>(L, out, bv, qp < MS_DESC_LDS ? L.msdesc[qp] : ms_desc(bv.ms + qp), qp, qm,
                             &L.bm[qm * T::MSTRIDE], L.nlen[qm], it.start,
                             ((uint64_t)it.k0_hi << 32) | it.k0_lo, it.k1, it.k2, it.k3, it.fmask);
      }
    }
    __syncthreads();  // the flush scratch aliases the bitmaps the decode reads
    PROF_ADD(12, t_dec);
  }
  if constexpr (LANE_MU) {  // finish every match of the tile: lane = match (message_unsynced.py:197-290)
    PROF_T(t_fin);
    {  // modulematch tables over the (now dead) decode queues. Loaded after the barrier on
       // purpose: values held in registers across it were parked in scratch by the compiler
       // (8.5 KB per tile written to and re-read from memory)
      const int m16 = (int)bv.hdr->mmtab_bytes >> 4;
      const uint4* msrc = reinterpret_cast<const uint4*>(bv.mmtab);
      uint4* mdst = reinterpret_cast<uint4*>(L.u.mmtab);
      for (int i = tid; i < m16; i += blockDim.x) mdst[i] = msrc[i];
      __syncthreads();
    }
    // matches past MATCH_CAP are in the spill region (a tile that overflowed is re-run: none then)
    const int nm = L.ovf ? 0 : (L.nmatch < MATCH_CAP + (int)SPILL_M ? L.nmatch : MATCH_CAP + (int)SPILL_M);
    const MuMatch* spilled = nm > MATCH_CAP ? reinterpret_cast<const MuMatch*>(out.work_dev + L.spill_base) : nullptr;
    // group the matches by protocol (counting sort into the free half of the queue region):
    // lanes of one wave then follow the same postDemod / modulematch / formatting path
    constexpr int NBIN = 256;
    static_assert(sizeof(L.u) >= SDX_MMTAB_LDS + MATCH_CAP * 2 + NBIN * 4, "sort scratch fits the union");
    uint16_t* perm = reinterpret_cast<uint16_t*>(L.u.mmtab + SDX_MMTAB_LDS);
    uint32_t* bin = reinterpret_cast<uint32_t*>(perm + MATCH_CAP);
    const bool sorted = (int)bv.hdr->n_mu <= NBIN && nm <= MATCH_CAP;
    if (sorted) {
      for (int i = tid; i < NBIN; i += blockDim.x) bin[i] = 0;
      __syncthreads();
      for (int m = tid; m < nm; m += blockDim.x) atomicAdd(&bin[L.mlist[m].p], 1u);
      __syncthreads();
      if (wave == 0) {  // exclusive prefix over the bins, 4 per lane
        uint32_t v[4], t = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = bin[4 * lane + k];
          t += v[k];
        }
        uint32_t x = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o);
          if (lane >= o) x += y;
        }
        uint32_t base = x - t;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          bin[4 * lane + k] = base;
          base += v[k];
        }
      }
      __syncthreads();
      for (int m = tid; m < nm; m += blockDim.x) perm[atomicAdd(&bin[L.mlist[m].p], 1u)] = (uint16_t)m;
      __syncthreads();
    }
    PROF_ADD(24, t_fin);
    PROF_T(t_fl0);
    // match i -> thread i: the first nm / 64 waves work, the others leave their SIMDs' issue slots
    // to the CU's other tile (contiguous blocks over all 8 waves measured slower: MU 1.144-1.159 vs
    // 1.124-1.125 ms, profiles/r03/s2/blk_*)
    for (int i = tid; i < nm; i += blockDim.x) {
      const MuMatch mm = i < MATCH_CAP ? L.mlist[sorted ? perm[i] : i] : spilled[i - MATCH_CAP];
      const int qm = mm.mi, qp = mm.p;
      const uint32_t rk = L.raise_key[qm];
      if (rk != 0xFFFFFFFFu && (rk >> 8) < (uint32_t)qp) continue;  // an earlier protocol raised
      sdx_mu_desc d;
      if (qp < SDX_MUDESC_LDS) d = L.desc[qp];
      else d = bv.mudesc[qp];
      const uint64_t* bmm = &L.bm[qm * T::MSTRIDE];
      M<NW> U, V1, VF;
      sym_masks<NW>(bmm, mm.u0, mm.u1, mm.u2, (mm.flags >> 3) & 7, d.width, &U, &V1, &VF);
      finish_mu_lane<NW>(L, out, wave, bv, bv.mu + qp, d, qp, qm, mm.j, mm.q, mm.k, d.width, (mm.flags & 1) != 0,
                         (uint8_t)((mm.flags >> 1) & 3), V1, VF);
    }
    PROF_ADD(25, t_fl0);
    PROF_T(t_fb);
    __syncthreads();
    PROF_ADD(26, t_fb);
    PROF_ADD(16, t_fin);
  }
  PROF_T(t_fl);
  flush_tile(L, msg_of, nvalid, out, bv, KIND);
  PROF_ADD(13, t_fl);
  PROF_ADD(15, t_kernel);
#ifdef SDX_WGTIME
  __syncthreads();
  if (tid == 0 && blk < 65536) g_wgt[2 * blk + 1] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef SDX_PROF
  if (lane < 28) atomicAdd(&g_prof[lane], (unsigned long long)L.prof[wave][lane]);
#endif
}

template <int KIND, int NW, int TM, int MR = 0, int SPLIT = 0>
__global__ __launch_bounds__((pulses_threads<KIND, NW>())) __attribute__((amdgpu_waves_per_eu(
    (NW <= 4 ? 4 : 1)))) void k_pulses(
    const void* __restrict__ bank, sdx_pulse_batch b, sdx_out out) {
  __shared__ PulsesLds<KIND, NW, TM> L;
  __shared__ int msg_of[TM];
  pulses_tile<KIND, NW, TM, MR, SPLIT>(bank, b, out, (int)blockIdx.x, L, msg_of);
}

// A copy on a few workgroups (sdx_copy_async_narrow): the streaming front end's device -> pinned-host
// result copies.  hipMemcpyAsync ran them as a blit kernel of 256 workgroups that held a slot on every CU
// for the whole PCIe transfer (0.4 ms per 500k-line chunk), beside the next chunks' demodulation
// tiles; this one holds nwg slots.  16-byte pieces when both ends are 16-byte aligned, bytes otherwise.
__global__ __launch_bounds__(256) void k_copy_narrow(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, size_t n) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  size_t done = 0;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15u) == 0) {
    const size_t n16 = n >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (size_t i = t; i < n16; i += 4 * nt) {  // four 16-byte pieces in flight per thread
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * nt < n16) v[u] = s4[i + u * nt];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * nt < n16) d4[i + u * nt] = v[u];
    }
    done = n16 << 4;
  }
  for (size_t i = done + t; i < n; i += nt) dst[i] = src[i];
}

// =============================================================================================
// MC engine (manchester.py "fixed" chain), lane = frame, 12 clockrange protocols uniform
// =============================================================================================
#ifndef SDX_STEP_ORDER
#define SDX_STEP_ORDER 0
#endif
#ifndef SDX_MS_TWO_LAUNCHES
#define SDX_MS_TWO_LAUNCHES 0
#endif
#ifndef SDX_MC_REC_CAP
#define SDX_MC_REC_CAP 152
#define SDX_MC_HEAP_CAP 3584
#endif
#ifndef SDX_MC_WPE
#define SDX_MC_WPE 4
#endif
// per wave: k_mc<4> fits 4 workgroups per CU (5 waves/SIMD with 96 / 2560 measured no faster:
// profiles/r05/dropped/time_mc5_*.log)
constexpr int MC_REC_CAP = SDX_MC_REC_CAP, MC_HEAP_CAP = SDX_MC_HEAP_CAP;

template <int MW>
struct McLds {
  uint64_t bn[MW * 256];   // bits, polarity as given
  uint64_t bi[MW * 256];   // bits, polarity inverted
  StageRec rec[4][MC_REC_CAP];
  alignas(16) uint8_t heap[4][MC_HEAP_CAP];
};

// a[w] <<= S bits across the MW-word bitstring (MSB-first words, 0 <= S < 64 * MW), no dynamic
// register indexing
template <int MW>
SDX_DEV void shl_words(uint64_t* a, int S) {
  const int q = S >> 6, r = S & 63;
  uint64_t o[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    uint64_t hi = 0, lo = 0;
#pragma unroll
    for (int k = 0; k < MW; ++k) {
      hi |= a[k] & (0ull - (uint64_t)(k == w + q));
      lo |= a[k] & (0ull - (uint64_t)(k == w + q + 1));
    }
    o[w] = r ? ((hi << r) | (lo >> (64 - r))) : hi;
  }
#pragma unroll
  for (int w = 0; w < MW; ++w) a[w] = o[w];
}

// hex -> MSB-first bits of a frame of 1..16 MW characters, both polarities, into the LDS words
// dn[w * 256] / di[w * 256] (helpers.py:168-188, manchester.py:36; leading zero nibbles dropped as
// bin(int(h, 16)) does, the last nibble always kept).  The characters come in with 2 MW + 1 aligned
// 8-byte loads issued together (hex_dev is readable 8 bytes past every frame's end) and are
// decoded in registers; the LDS words are written once.
template <int MW>
SDX_DEV void mc_stage(const uint8_t* src, int hl, uint64_t* dn, uint64_t* di, int* nN, int* nI, bool* ok) {
  constexpr int NR = 2 * MW + 1;
  const int s = (int)((uintptr_t)src & 7);
  const uint64_t* wp = reinterpret_cast<const uint64_t*>(src - s);
  uint64_t raw[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) raw[k] = (8 * k < s + hl) ? wp[k] : 0ull;
  uint64_t wn[MW], wi[MW];
#pragma unroll
  for (int w = 0; w < MW; ++w) wn[w] = wi[w] = 0;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 2 * MW; ++k) {
    const uint64_t x = s ? ((raw[k] >> (8 * s)) | (raw[k + 1] << (64 - 8 * s))) : raw[k];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = 8 * k + j;
      const uint32_t c = (uint32_t)(x >> (8 * j)) & 0xFFu;
      const bool in = i < hl;
      const bool dig = c - '0' < 10u, up = c - 'A' < 6u, lo = c - 'a' < 6u;
      bad |= in && !(dig || up || lo);
      const uint32_t v = dig ? c - '0' : (c & 7u) + 9u;  // 'A'/'a' -> 10 ... 'F'/'f' -> 15
      const uint32_t vi = (dig || up) ? 15u - v : v;      // str.translate: uppercase only
      const int sh = 60 - 4 * (i & 15);
      wn[i >> 4] |= (uint64_t)(in ? v & 15u : 0u) << sh;
      wi[i >> 4] |= (uint64_t)(in ? vi & 15u : 0u) << sh;
    }
  }
  *ok = !bad;
  // leading zero nibbles (at most hl - 1 of them)
  auto lead = [&](const uint64_t* a) -> int {
    int f = 64 * MW;
#pragma unroll
    for (int w = MW - 1; w >= 0; --w)
      if (a[w]) f = 64 * w + __clzll((long long)a[w]);
    const int lz = f >> 2;
    return lz < hl - 1 ? lz : hl - 1;
  };
  const int lzn = lead(wn), lzi = lead(wi);
  shl_words<MW>(wn, 4 * lzn);
  shl_words<MW>(wi, 4 * lzi);
  *nN = 4 * (hl - lzn);
  *nI = 4 * (hl - lzi);
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    dn[w * 256] = wn[w];
    di[w * 256] = wi[w];
  }
}

// MW = 4: frames of <= 64 hex characters, longer ones are left to the MW = 8 launch (LONG = true),
// which takes only those (sdx_demod_mc launches both; a wave without long frames exits at once)
// 256 frames (blk = the block's index in the launch, tid = 0..255 the frame's thread) of a k_mc
// launch; the LDS comes from the calling kernel (k_mc, or one half of a k_step block)
template <int MW, bool LONG>
SDX_DEV void mc_block(const void* __restrict__ bank, const sdx_mc_batch& b, const sdx_out& out, const int blk,
                      const int tid, McLds<MW>& L) {
  const BankView bv = bank_view(bank);
  const int wave = tid >> 6, lane = tid & 63;
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int gi = blk * 256 + tid;
  bool valid = gi < ntot;
  const int msg = valid ? (b.sel_dev ? b.sel_dev[gi] : gi) : 0;
  bool toolong = false;  // > MC_MAXW * 16 characters: left to sdx_demod_mc_general (status OVF_TILE)
  if (valid) {  // this launch's share: short frames (MW = 4) or long ones
    const int hl0 = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - b.offsets_dev[msg]);
    valid = LONG ? hl0 > MC_SHORTW * 16 : hl0 <= MC_SHORTW * 16;
    if (LONG && valid && hl0 > MW * 16) {
      toolong = true;
      valid = false;
    }
    // a frame longer than the batch's promised bound (0 < max_hex <= 64: no long launch follows) is
    // marked for a re-run instead of being left without a descriptor
    if (!LONG && !valid && b.max_hex > 0 && b.max_hex <= MC_SHORTW * 16) toolong = true;
  }
  if (toolong) {
    sdx_desc d;
    d.rec_begin = 0;
    d.n_rec = 0;
    d.status = SDX_ST_OVF_TILE;
    d.raise_kind = 0;
    out.desc_dev[msg] = d;
    atomicOr(&out.cursor_dev[2], 2u);
  }
  if (LONG && !__ballot(valid)) return;  // whole wave without long frames (nothing staged yet)
#ifdef SDX_PROF  // per-wave cycles of k_mc's phases (g_prof slots 27-31, tools/prof_phases.py), summed
  // in registers; per protocol (g_gprof[0][p] cycles, [1][p] lanes through the gates) in LDS
  unsigned long long mcacc[5] = {0, 0, 0, 0, 0};
  __shared__ unsigned long long mcp[2][32];
  if (tid < 64) mcp[tid >> 5][tid & 31] = 0;
  if constexpr (!LONG) __syncthreads();
#define MCPROF_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define MCPROF_ADD(slot, v) mcacc[(slot) - 27] += __builtin_amdgcn_s_memtime() - (v)
#else
#define MCPROF_T(v)
#define MCPROF_ADD(slot, v)
#endif
  MCPROF_T(t_all);
  MCPROF_T(t_st);
  int w_heap = 0, w_rec = 0;  // the wave's staged payload bytes and records (wave-uniform)
  bool w_ovf = false;
  const LaneBits BN{&L.bn[tid], MW, false}, BI{&L.bi[tid], MW, false};
  // hex -> bits for both polarities (helpers.py:168-188: leading zero nibbles are dropped)
  int nN = 0, nI = 0;
  bool hex_ok = false;
  int clock = 0, mcbit = 0, flags = 0, only = -1;
  if (valid) {
    const int64_t off = b.offsets_dev[msg];
    const int hl = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
    clock = b.clock_dev[msg];
    mcbit = b.mcbitnum_dev[msg];
    flags = b.flags_dev[msg];
    if (b.only_dev) only = b.only_dev[msg];
    hex_ok = hl > 0 && hl <= MW * 16;
    if (hex_ok) mc_stage<MW>(b.hex_dev + off, hl, &L.bn[tid], &L.bi[tid], &nN, &nI, &hex_ok);
  }
  MCPROF_ADD(27, t_st);
  const int nmc = (int)bv.hdr->n_mc;
  int raise = 0, mycnt = 0;
  for (int p = 0; p < nmc; ++p) {
    MCPROF_T(t_m);
    const sdx_mc_proto* r = uniform_ptr(bv.mc + p);
    bool go = valid && !raise && (only < 0 || only == p);
    // gates of _demodulate_mc_data (manchester.py:70-89; clockrange fixed to [0] / [1])
    if (go && mcbit < (cld(&r->has_lmin) ? cld(&r->lmin) : -1)) go = false;
    if (go && mcbit > (cld(&r->has_lmax) ? cld(&r->lmax) : 9999)) go = false;
    if (go && cld(&r->has_cr) && !((double)clock > cld(&r->cr_lo) && (double)clock < cld(&r->cr_hi))) go = false;
    McOut o{0, 0, 0, 0, 0, 0, 0, 0};
    const bool inv = (cld(&r->invert) != 0) ^ ((flags & 3) != 0);  // (:91-96)
    const LaneBits& B = inv ? BI : BN;
    const int nb = inv ? nI : nN;
    if (go && !hex_ok) { raise = SDX_RAISE_TYPE; go = false; }  // len(None) -> TypeError
    if (go) {
      const LaneBits DM{B.base, MW, true};  // mc2dmc(lh/hl) view for Funkbus
      o = mc_method(r, cld(&r->method), B, nb, nb, DM);
      if (o.rc == -1) { raise = SDX_RAISE_TYPE; o.rc = 0; }
      if (o.rc == -2) { raise = SDX_RAISE_VALUE; o.rc = 0; }
    }
    // stage results of the wave in lane (= frame) order for this protocol
    const bool has = o.rc == 1;
    MCPROF_ADD(28, t_m);
#ifdef SDX_PROF
    if (lane == 0 && p < 32) {
      atomicAdd(&mcp[0][p], __builtin_amdgcn_s_memtime() - t_m);
      atomicAdd(&mcp[1][p], (unsigned long long)__popcll(ballot(go)));
    }
#endif
    if (!ballot(has)) continue;  // no result in this wave: nothing to stage (wave-uniform)
    MCPROF_T(t_r);
    const int plen = has ? cld(&r->pre_len) + o.len : 0;
    int incl = plen;  // inclusive scan over lanes
    for (int d = 1; d < WAVE; d <<= 1) {
      const int t = __shfl_up(incl, d);
      if (lane >= d) incl += t;
    }
    const int wtot = __shfl(incl, WAVE - 1);
    const uint64_t hm = ballot(has);
    const int nnew = popc64(hm);
    const int hb = w_heap, rb = w_rec;
    const bool fits = hb + wtot <= MC_HEAP_CAP && rb + nnew <= MC_REC_CAP;
    if (has && fits) {
      uint8_t* dst = &L.heap[wave][hb + incl - plen];
      const int pl = cld(&r->pre_len), po = cld(&r->pre_off);
      for (int i = 0; i < pl; i += 8) {  // 8 independent loads per step
        uint8_t c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = (i + j < pl) ? bv.str[po + i + j] : (uint8_t)0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (i + j < pl) dst[i + j] = c[j];
      }
      mc_write(r, o, B, nb, nb, dst + cld(&r->pre_len));
      StageRec sr;
      sr.off = (uint32_t)(hb + incl - plen);
      sr.len = (uint16_t)plen;
      sr.proto = (uint16_t)p;
      sr.bitlen = 0;
      sr.msg = (uint16_t)lane;
      sr.rank = (uint16_t)mycnt;  // this frame's records so far (protocol order)
      L.rec[wave][rb + lanes_below(hm)] = sr;
      ++mycnt;
    }
    if (fits) {  // the wave's staging cursors are wave-uniform registers (every lane computes them)
      w_heap = hb + wtot;
      w_rec = rb + nnew;
    } else if (nnew) {
      w_ovf = true;
    }
    MCPROF_ADD(29, t_r);
  }
  wave_sync();  // the staged records and payloads of all lanes, for the flush
  MCPROF_T(t_f);
  // flush this wave's frames: records are staged in protocol-major order, each carrying its rank
  // among its frame's records; the wave writes them 64 at a time to (frame, protocol) order
  const int nr = w_rec;
  const int nh = (w_heap + 15) & ~15;  // 16-B pieces: every reservation keeps hbase aligned
  const bool bad = w_ovf;
  if (raise) mycnt = 0;
  int incl = mycnt;
  for (int d = 1; d < WAVE; d <<= 1) {
    const int t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  const int wrec = __shfl(incl, WAVE - 1);
  uint32_t rbase = 0, hbase = 0;
  int st = bad ? 2 : 0;
  if (lane == 0 && !bad) {
    rbase = atomicAdd(&out.cursor_dev[0], (uint32_t)wrec);
    hbase = atomicAdd(&out.cursor_dev[1], (uint32_t)nh);
    if (rbase + wrec > out.rec_cap || hbase + nh > out.heap_cap) { st = 3; atomicOr(&out.cursor_dev[2], 1u); }
  }
  if (lane == 0 && bad) atomicOr(&out.cursor_dev[2], 2u);
  rbase = (uint32_t)__shfl((int)rbase, 0);
  hbase = (uint32_t)__shfl((int)hbase, 0);
  st = __shfl(st, 0);
  // the exchange's counts (ABI 12): per frame payload << 32 | wire bytes, in this wave's slice of
  // the (now dead) bit rows
  const bool wx = out.wire_dev != nullptr;
  unsigned long long* wsum = reinterpret_cast<unsigned long long*>(&L.bn[64 * wave]);
  if (wx) {
    wsum[lane] = 0ull;
    wave_sync();
  }
  if (st == 0) {
    const int excl = incl - mycnt;
    for (int i0 = 0; i0 < nr; i0 += WAVE) {  // wave-uniform trip count (the shuffles below)
      const int i = i0 + lane;
      StageRec sr{};
      if (i < nr) sr = L.rec[wave][i];
      const int fl = i < nr ? (int)sr.msg : 0;
      const int fbase = __shfl(excl, fl), fmsg = __shfl(msg, fl), fraise = __shfl(raise, fl);
      if (i < nr && !fraise) {
        sdx_result o;
        o.payload_off = hbase + sr.off;
        o.payload_len = sr.len;
        o.proto = sr.proto;
        o.bit_length = 0;
        o.msg = (uint32_t)fmsg;
        out.rec_dev[rbase + fbase + sr.rank] = o;
        if (wx) {
          const uint32_t xr = wire_class(bv, SDX_KIND_MC, sr.proto, &L.heap[wave][sr.off], sr.len);
          if (out.xrec_dev) out.xrec_dev[rbase + fbase + sr.rank] = xr;
          atomicAdd(&wsum[fl], (unsigned long long)(((uint64_t)sr.len << 32) | wire_bytes_x(xr, sr.len)));
        }
      }
    }
    uint4* hd = reinterpret_cast<uint4*>(out.heap_dev + hbase);
    const uint4* hs = reinterpret_cast<const uint4*>(L.heap[wave]);
    if ((((uintptr_t)hd) & 15u) == 0) {
      for (int i = lane; i < (nh >> 4); i += WAVE) hd[i] = hs[i];
    } else {
      for (int i = lane; i < nh; i += WAVE) out.heap_dev[hbase + i] = L.heap[wave][i];
    }
  }
  if (valid) {
    sdx_desc d;
    d.rec_begin = rbase + (uint32_t)(incl - mycnt);
    if (raise) { d.status = SDX_ST_RAISED; d.raise_kind = (uint8_t)raise; d.n_rec = 0; }
    else if (st) { d.status = st == 2 ? SDX_ST_OVF_TILE : SDX_ST_OVF_OUT; d.raise_kind = 0; d.n_rec = 0; }
    else { d.status = SDX_ST_OK; d.raise_kind = 0; d.n_rec = (uint16_t)mycnt; }
    out.desc_dev[msg] = d;
  }
  if (wx) {
    wave_sync();
    if (valid) out.wire_dev[msg] = (!raise && st == 0) ? (uint64_t)wsum[lane] : 0ull;
  }
  MCPROF_ADD(30, t_f);
  MCPROF_ADD(31, t_all);
#ifdef SDX_PROF
  if (lane == 0)
    for (int i = 0; i < 5; ++i) atomicAdd(&g_prof[27 + i], mcacc[i]);
  if constexpr (!LONG) {
    __syncthreads();
    if (tid < 64) atomicAdd(&g_gprof[tid >> 5][tid & 31], mcp[tid >> 5][tid & 31]);
  }
#endif
#undef MCPROF_T
#undef MCPROF_ADD
}

// ---------------------------------------------------------------------------------------------
// compacted MC block (frames of <= 64 characters).  mc_block runs every protocol on
// every wave: per (wave, protocol) the method and the result staging execute for the ~4 of 64 lanes
// whose frame passed the protocol's gates, i.e. 4 waves x 12 protocols of mostly idle method passes
// (measured: the methods + staging are 0.15 of k_mc's 0.18 ms; gates alone 0.03 ms).  Here the gates
// run lane = frame and leave a 12-bit mask per frame; then each wave takes whole protocols (an LDS
// counter) and runs the method over the frames of the WHOLE block that passed that protocol's gates,
// compacted 64 to a pass -- the protocol stays wave-uniform (scalar record loads, mc_method as is) --
// staging into block-wide pools; a block-level flush places the records in (frame, protocol) order.
// Results, statuses and raise kinds are the per-frame sequential loop's: a frame raises with the kind
// of the FIRST protocol (bank order) that raises for it, and then publishes nothing.
// ---------------------------------------------------------------------------------------------
constexpr int MC_BREC = 512, MC_BHEAP = 11264;  // block-wide staging pools (bench mean ~97 records,
                                                 // ~2.9 KB of payload per 256 frames)
constexpr int MC_CMAXP = 16;                      // protocols of the gate mask (the bank has 12)
constexpr uint32_t MC_NORAISE = 0xFFFFFFFFu;
template <int MW>
struct McLdsC {
  uint64_t bn[MW * 256];   // bits, polarity as given
  uint64_t bi[MW * 256];   // bits, polarity inverted
  StageRec rec[MC_BREC];
  alignas(16) uint8_t heap[MC_BHEAP];
  uint16_t gm[256];        // bit p: the frame passed protocol p's gates (and is valid hex)
  uint16_t nbits[2][256];  // len(bits) as given / inverted (leading zero nibbles dropped)
  uint8_t fl[256];         // the frame's flags (bits 0-1: message type / version)
  uint8_t list[4][256];    // per wave: the frames of the protocol it runs
  uint32_t fraise[256];    // p << 4 | kind of the first raising protocol (bank order), MC_NORAISE: none
  uint32_t rcur, hcur, pnext, ovf;
};

template <int MW>
SDX_DEV void mc_block_c(const void* __restrict__ bank, const sdx_mc_batch& b, const sdx_out& out, const int blk,
                        const int tid, McLdsC<MW>& L) {
  const BankView bv = bank_view(bank);
  const int wave = tid >> 6, lane = tid & 63;
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int gi = blk * 256 + tid;
  bool valid = gi < ntot;
  const int msg = valid ? (b.sel_dev ? b.sel_dev[gi] : gi) : 0;
  const int nmc = (int)bv.hdr->n_mc;
  if (tid == 0) {
    L.rcur = 0;
    L.hcur = 0;
    L.pnext = 0;
    L.ovf = 0;
  }
  // ---- lane = frame: this launch's share, hex -> bits (both polarities), the gates of every protocol
  bool toolong = false;
  if (valid) {
    const int hl0 = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - b.offsets_dev[msg]);
    valid = hl0 <= MC_SHORTW * 16;
    // a frame longer than the batch's promised bound (0 < max_hex <= 64: no long launch follows) is
    // marked for a re-run instead of being left without a descriptor
    if (!valid && b.max_hex > 0 && b.max_hex <= MC_SHORTW * 16) toolong = true;
  }
  if (toolong) {
    sdx_desc d;
    d.rec_begin = 0;
    d.n_rec = 0;
    d.status = SDX_ST_OVF_TILE;
    d.raise_kind = 0;
    out.desc_dev[msg] = d;
    atomicOr(&out.cursor_dev[2], 2u);
  }
  int nN = 0, nI = 0;
  bool hex_ok = false;
  int clock = 0, mcbit = 0, flags = 0, only = -1;
  if (valid) {
    const int64_t off = b.offsets_dev[msg];
    const int hl = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
    clock = b.clock_dev[msg];
    mcbit = b.mcbitnum_dev[msg];
    flags = b.flags_dev[msg];
    if (b.only_dev) only = b.only_dev[msg];
    hex_ok = hl > 0 && hl <= MW * 16;
    if (hex_ok) mc_stage<MW>(b.hex_dev + off, hl, &L.bn[tid], &L.bi[tid], &nN, &nI, &hex_ok);
  }
  // gates of _demodulate_mc_data (manchester.py:70-89; clockrange fixed to [0] / [1])
  uint32_t gm = 0;
  for (int p = 0; p < nmc; ++p) {
    const sdx_mc_proto* r = uniform_ptr(bv.mc + p);
    bool go = valid && (only < 0 || only == p);
    if (go && mcbit < (cld(&r->has_lmin) ? cld(&r->lmin) : -1)) go = false;
    if (go && mcbit > (cld(&r->has_lmax) ? cld(&r->lmax) : 9999)) go = false;
    if (go && cld(&r->has_cr) && !((double)clock > cld(&r->cr_lo) && (double)clock < cld(&r->cr_hi))) go = false;
    gm |= (uint32_t)go << p;
  }
  // a frame that is not valid hex raises at its first protocol past the gates (len(None) -> TypeError)
  // and runs no method
  const uint32_t r0 = (gm && !hex_ok) ? (((uint32_t)(__ffs(gm) - 1) << 4) | SDX_RAISE_TYPE) : MC_NORAISE;
  L.gm[tid] = hex_ok ? (uint16_t)gm : (uint16_t)0;
  L.nbits[0][tid] = (uint16_t)nN;
  L.nbits[1][tid] = (uint16_t)nI;
  L.fl[tid] = (uint8_t)(flags & 3);
  L.fraise[tid] = r0;
  __syncthreads();
  // ---- per wave: whole protocols, each over the block's frames that passed its gates, 64 per pass
  for (;;) {
    int p = 0;
    if (lane == 0) p = (int)atomicAdd(&L.pnext, 1u);
    p = __shfl(p, 0);
    if (p >= nmc) break;
    const sdx_mc_proto* r = uniform_ptr(bv.mc + p);
    int cnt = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f = g * 64 + lane;
      const bool on = (L.gm[f] >> p) & 1u;
      const uint64_t m = ballot(on);
      if (on) L.list[wave][cnt + lanes_below(m)] = (uint8_t)f;
      cnt += popc64(m);
    }
    wave_sync();
    const bool pinv = cld(&r->invert) != 0;
    const int method = cld(&r->method);
    const int pl = cld(&r->pre_len), po = cld(&r->pre_off);
    for (int i0 = 0; i0 < cnt; i0 += WAVE) {
      const int i = i0 + lane;
      const bool act = i < cnt;
      const int f = act ? (int)L.list[wave][i] : 0;
      const bool inv = pinv ^ (L.fl[f] != 0);  // (:91-96)
      const LaneBits BN{&L.bn[f], MW, false}, BI{&L.bi[f], MW, false};
      const LaneBits& B = inv ? BI : BN;
      const int nb = L.nbits[inv ? 1 : 0][f];
      McOut o{0, 0, 0, 0, 0, 0, 0, 0};
      if (act) {
        const LaneBits DM{B.base, MW, true};  // mc2dmc(lh/hl) view for Funkbus
        o = mc_method(r, method, B, nb, nb, DM);
        int rk = 0;
        if (o.rc == -1) { rk = SDX_RAISE_TYPE; o.rc = 0; }
        if (o.rc == -2) { rk = SDX_RAISE_VALUE; o.rc = 0; }
        if (rk) atomicMin(&L.fraise[f], ((uint32_t)p << 4) | (uint32_t)rk);  // the first raising protocol
      }
      const bool has = o.rc == 1;
      const uint64_t hm = ballot(has);
      if (!hm) continue;
      const int plen = has ? pl + o.len : 0;
      int incl = plen;  // inclusive scan over lanes
      for (int d = 1; d < WAVE; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
      }
      const int wtot = __shfl(incl, WAVE - 1);
      const int nnew = popc64(hm);
      uint32_t hb = 0, rb = 0;
      if (lane == 0) {
        hb = atomicAdd(&L.hcur, (uint32_t)wtot);
        rb = atomicAdd(&L.rcur, (uint32_t)nnew);
      }
      hb = (uint32_t)__shfl((int)hb, 0);
      rb = (uint32_t)__shfl((int)rb, 0);
      const bool fits = hb + (uint32_t)wtot <= (uint32_t)MC_BHEAP && rb + (uint32_t)nnew <= (uint32_t)MC_BREC;
      if (!fits) {
        if (lane == 0) L.ovf = 1u;
        continue;
      }
      if (has) {
        uint8_t* dst = &L.heap[hb + incl - plen];
        for (int k = 0; k < pl; k += 8) {  // 8 independent loads per step
          uint8_t c[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) c[j] = (k + j < pl) ? bv.str[po + k + j] : (uint8_t)0;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (k + j < pl) dst[k + j] = c[j];
        }
        mc_write(r, o, B, nb, nb, dst + pl);
        StageRec sr;
        sr.off = hb + (uint32_t)(incl - plen);
        sr.len = (uint16_t)plen;
        sr.proto = (uint16_t)p;
        sr.bitlen = 0;
        sr.msg = (uint8_t)f;
        sr.wave = 0;
        sr.rank = 0;
        L.rec[rb + lanes_below(hm)] = sr;
      }
    }
  }
  __syncthreads();
  // ---- block flush: records bucketed by frame, each frame's in protocol order (flush_tile's scheme)
  const int nr = (int)(L.rcur < (uint32_t)MC_BREC ? L.rcur : (uint32_t)MC_BREC);
  const int nh = (int)(((L.hcur < (uint32_t)MC_BHEAP ? L.hcur : (uint32_t)MC_BHEAP) + 15u) & ~15u);
  const bool bad = L.ovf != 0;
  // scratch in the (dead) bit rows: per frame the record count, bucket fill, base, wire sums; the
  // bucketed record indices
  uint32_t* cntm = reinterpret_cast<uint32_t*>(L.bn);
  uint32_t* fill = cntm + 256;
  uint32_t* mbase = fill + 256;
  uint32_t* wtot = mbase + 256;      // [4] per wave totals of the scan, [4..5] rbase / hbase, [6] st
  unsigned long long* wsum = reinterpret_cast<unsigned long long*>(L.bi);
  uint16_t* bidx = reinterpret_cast<uint16_t*>(wsum + 256);
  static_assert(4 * (3 * 256 + 8) <= (int)sizeof(L.bn) && 8 * 256 + 2 * MC_BREC <= (int)sizeof(L.bi), "flush scratch");
  const bool raised = L.fraise[tid] != MC_NORAISE;
  cntm[tid] = 0;
  fill[tid] = 0;
  wsum[tid] = 0ull;
  __syncthreads();
  if (!bad)
    for (int k = tid; k < nr; k += 256) {
      const int f = L.rec[k].msg;
      if (L.fraise[f] == MC_NORAISE) atomicAdd(&cntm[f], 1u);
    }
  __syncthreads();
  // exclusive scan of the 256 counts (lane = frame): wave scans + the waves' totals
  const uint32_t c = (valid && !raised && !bad) ? cntm[tid] : 0u;
  uint32_t x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wtot[wave] = x;
  __syncthreads();
  uint32_t before = 0;
  for (int w = 0; w < wave; ++w) before += wtot[w];
  mbase[tid] = before + x - c;
  if (tid == 0) {
    const uint32_t nrec = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    uint32_t st = bad ? 2u : 0u, rbase = 0, hbase = 0;
    if (!bad) {
      rbase = atomicAdd(&out.cursor_dev[0], nrec);
      hbase = atomicAdd(&out.cursor_dev[1], (uint32_t)nh);
      if (rbase + nrec > out.rec_cap || hbase + (uint32_t)nh > out.heap_cap) {
        st = 3u;
        atomicOr(&out.cursor_dev[2], 1u);
      }
    } else {
      atomicOr(&out.cursor_dev[2], 2u);
    }
    wtot[4] = rbase;
    wtot[5] = hbase;
    wtot[6] = st;
    wtot[7] = nrec;
  }
  __syncthreads();
  const uint32_t rbase = wtot[4], hbase = wtot[5], st = wtot[6], nrec = wtot[7];
  const bool wx = out.wire_dev != nullptr;
  if (st == 0) {
    for (int k = tid; k < nr; k += 256) {
      const int f = L.rec[k].msg;
      if (L.fraise[f] != MC_NORAISE) continue;
      const uint32_t q = atomicAdd(&fill[f], 1u);
      bidx[mbase[f] + q] = (uint16_t)k;
    }
    __syncthreads();
    for (int j = tid; j < (int)nrec; j += 256) {
      const StageRec sr = L.rec[bidx[j]];
      const uint32_t b0 = mbase[sr.msg], b1 = b0 + cntm[sr.msg];
      uint32_t rk = 0;  // one record per (frame, protocol): its rank = the frame's records of lower protocols
      for (uint32_t q = b0; q < b1; ++q) rk += L.rec[bidx[q]].proto < sr.proto ? 1u : 0u;
      const int gf = blk * 256 + sr.msg;
      sdx_result o;
      o.payload_off = hbase + sr.off;
      o.payload_len = sr.len;
      o.proto = sr.proto;
      o.bit_length = 0;
      o.msg = (uint32_t)(b.sel_dev ? b.sel_dev[gf] : gf);
      out.rec_dev[rbase + b0 + rk] = o;
      if (wx) {
        const uint32_t xr = wire_class(bv, SDX_KIND_MC, sr.proto, &L.heap[sr.off], sr.len);
        if (out.xrec_dev) out.xrec_dev[rbase + b0 + rk] = xr;
        atomicAdd(&wsum[sr.msg], (unsigned long long)(((uint64_t)sr.len << 32) | wire_bytes_x(xr, sr.len)));
      }
    }
    uint4* hd = reinterpret_cast<uint4*>(out.heap_dev + hbase);
    const uint4* hs = reinterpret_cast<const uint4*>(L.heap);
    if ((((uintptr_t)hd) & 15u) == 0) {
      for (int k = tid; k < (nh >> 4); k += 256) hd[k] = hs[k];
    } else {
      for (int k = tid; k < nh; k += 256) out.heap_dev[hbase + k] = L.heap[k];
    }
  }
  if (wx) __syncthreads();  // wsum complete
  if (valid) {
    sdx_desc d;
    d.rec_begin = rbase + mbase[tid];
    const uint32_t rw = L.fraise[tid];
    if (rw != MC_NORAISE) { d.status = SDX_ST_RAISED; d.raise_kind = (uint8_t)(rw & 15u); d.n_rec = 0; }
    else if (st) { d.status = st == 2 ? SDX_ST_OVF_TILE : SDX_ST_OVF_OUT; d.raise_kind = 0; d.n_rec = 0; }
    else { d.status = SDX_ST_OK; d.raise_kind = 0; d.n_rec = (uint16_t)cntm[tid]; }
    out.desc_dev[msg] = d;
    if (wx) out.wire_dev[msg] = (rw == MC_NORAISE && st == 0) ? (uint64_t)wsum[tid] : 0ull;
  }
}

template <int MW, bool LONG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LONG ? 1 : SDX_MC_WPE))) void k_mc(const void* __restrict__ bank, sdx_mc_batch b, sdx_out out) {
  if constexpr (LONG) {
    __shared__ McLds<MW> L;
    mc_block<MW, LONG>(bank, b, out, (int)blockIdx.x, (int)threadIdx.x, L);
  } else {
    __shared__ McLdsC<MW> L;
    mc_block_c<MW>(bank, b, out, (int)blockIdx.x, (int)threadIdx.x, L);
  }
}

// ---------------------------------------------------------------------------------------------
// k_step: a mixed step's MU, MS and MC launches as one grid (sdx_demod_step).  Workgroups are
// dispatched in index order, so MU's tiles go first, then MS's (each tile on the instantiation of its
// length class, NW = 2 when no message has more than 128 pulses), then MC's frames, two 256-frame
// blocks per workgroup.  A kind's tiles start on the CU slots the previous kind's last tiles
// free: with one launch per kind, each launch's tail (its last round of tiles finishing unevenly)
// idled the CUs until the whole launch had ended.  One LDS union serves every kind (the MU tile is the
// largest at 80.7 KB; two MC blocks 80.9 KB) and every body fits the MU tile's 128 VGPRs, so each kind
// keeps its own occupancy (2 tiles per CU).
// ---------------------------------------------------------------------------------------------
// one MS tile on the instantiation of its length class: NW = 2 (2 bitmap words per id, 118 VGPRs)
// when none of its messages has more than 128 pulses, NW = 4 otherwise -- decided per tile, so no
// workgroup exists only to find that the tile is another launch's.  MR = 1: the header fields (and the
// length deciding the class) from the message records the grouping wrote (one 128-byte line per
// message instead of a sector of each SoA field)
template <int MR>
SDX_DEV void ms_tile_by_class(const void* __restrict__ bank, const sdx_pulse_batch& b, const sdx_out& out, const int w,
                              PulsesLds<SDX_KIND_MS, 2, 64>& L2, PulsesLds<SDX_KIND_MS, 4, 64>& L4, int* msg_of) {
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int m = w * 64 + (int)threadIdx.x;
  int len = 0;
  if (threadIdx.x < 64 && m < ntot) {
    const int msg = b.sel_dev ? b.sel_dev[m] : m;
    if (MR)
      len = b.mrec_dev[msg].len;
    else
      len = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - b.offsets_dev[msg]);
  }
  if (__syncthreads_or(len > 128) == 0)
    pulses_tile<SDX_KIND_MS, 2, 64, MR, 0>(bank, b, out, w, L2, msg_of);
  else
    pulses_tile<SDX_KIND_MS, 4, 64, MR, 0>(bank, b, out, w, L4, msg_of);
}

// sdx_demod_pulses(MS): every tile on its length class's instantiation
template <int MR>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_ms_classes(
    const void* __restrict__ bank, sdx_pulse_batch b, sdx_out out) {
  __shared__ union {
    PulsesLds<SDX_KIND_MS, 2, 64> n2;
    PulsesLds<SDX_KIND_MS, 4, 64> n4;
  } U;
  __shared__ int msg_of[64];
  ms_tile_by_class<MR>(bank, b, out, (int)blockIdx.x, U.n2, U.n4, msg_of);
}

struct StepArgs {
  sdx_pulse_batch mu, ms;
  sdx_mc_batch mc;
  sdx_out mu_out, ms_out, mc_out;
  int t_mu, t_ms, b_mc;  // workgroups of each range (b_mc: pairs of 256-frame blocks)
};
union StepLds {
  PulsesLds<SDX_KIND_MU, 4, 64> mu;
  PulsesLds<SDX_KIND_MS, 2, 64> ms2;
  PulsesLds<SDX_KIND_MS, 4, 64> ms4;
  McLdsC<MC_SHORTW> mc[2];
};
static_assert(sizeof(StepLds) <= 81920, "two k_step workgroups per CU (160 KB of LDS)");

template <int MRU, int MRS>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_step(const void* __restrict__ bank,
                                                                                      StepArgs a) {
  static_assert(pulses_threads<SDX_KIND_MU, 4>() == 512 && pulses_threads<SDX_KIND_MS, 2>() == 512, "512-thread tiles");
  __shared__ StepLds U;
  __shared__ int msg_of[64];
  // the ranges in dispatch order (SDX_STEP_ORDER): 0 = MU, MS, MC; 1 = MC, MU, MS; 2 = MU, MC, MS
  constexpr int R0 = SDX_STEP_ORDER == 0 ? 0 : (SDX_STEP_ORDER == 1 ? 2 : 0);
  constexpr int R1 = SDX_STEP_ORDER == 0 ? 1 : (SDX_STEP_ORDER == 1 ? 0 : 2);
  constexpr int R2 = SDX_STEP_ORDER == 0 ? 2 : 1;
  const int cnt[3] = {a.t_mu, a.t_ms, a.b_mc};
  int w = (int)blockIdx.x, r = R2;
  if (w < cnt[R0]) {
    r = R0;
  } else {
    w -= cnt[R0];
    if (w < cnt[R1]) r = R1;
    else w -= cnt[R1];
  }
  if (r == 0) {
    pulses_tile<SDX_KIND_MU, 4, 64, MRU, 0>(bank, a.mu, a.mu_out, w, U.mu, msg_of);
  } else if (r == 1) {
    ms_tile_by_class<MRS>(bank, a.ms, a.ms_out, w, U.ms2, U.ms4, msg_of);
  } else {
    const int half = (int)threadIdx.x >> 8;
    mc_block_c<MC_SHORTW>(bank, a.mc, a.mc_out, 2 * w + half, (int)threadIdx.x & 255, U.mc[half]);
  }
}

}  // namespace sdx

// =============================================================================================
// C-ABI
// =============================================================================================
struct sdx_bank {
  int device;
  void* dev;
  size_t nbytes;
  sdx_bank_hdr hdr;
};

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
namespace sdx {
size_t group_bytes(int n);  // sdx_group.hip
bool group_messages(const void* bank_dev, int kind, const sdx_pulse_batch& b, int32_t* order, sdx_msg_rec* mrec, uint8_t* work,
                    size_t bytes, hipStream_t st);
bool group_messages2(const void* bank_dev, const sdx_pulse_batch& bmu, int32_t* omu, sdx_msg_rec* rmu, uint8_t* wmu,
                     size_t cmu, const sdx_pulse_batch& bms, int32_t* oms, sdx_msg_rec* rms, uint8_t* wms, size_t cms,
                     hipStream_t st);
// for the other translation units (sdx_lines.hip, sdx_mn.hip): the error text of sdx_last_error()
// and the bank handle's fields
int set_error(int code, const std::string& msg) { return fail(code, msg); }
const void* bank_dev_ptr(const sdx_bank* b) { return b->dev; }
const sdx_bank_hdr* bank_hdr(const sdx_bank* b) { return &b->hdr; }
}  // namespace sdx
#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return fail(SDX_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

extern "C" {

int sdx_abi_version(void) { return SDX_ABI_VERSION; }

#ifdef SDX_PROF
int sdx_gprof_read(unsigned long long* out256, int reset) {
  HIPCHK(hipMemcpyFromSymbol(out256, HIP_SYMBOL(g_gprof), sizeof(unsigned long long) * 256));
  if (reset) {
    unsigned long long z[256] = {0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_gprof), z, sizeof z));
  }
  return SDX_OK;
}
int sdx_prof_read(unsigned long long* out32, int reset) {
  HIPCHK(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 32));
  if (reset) {
    unsigned long long z[32] = {0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z));
  }
  return SDX_OK;
}
#endif
#ifdef SDX_WGTIME
int sdx_wgtime_read(unsigned long long* out, int n) {
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wgt), sizeof(unsigned long long) * 2 * (n < 65536 ? n : 65536)));
  return SDX_OK;
}
#endif
const char* sdx_last_error(void) { return g_err.c_str(); }

// sdx_source_hash(): defined in the build's generated translation unit (build.py, _lib/obj/sdx_hash.cpp),
// so a change of one source recompiles only that source

int sdx_layout_size(int which) {
  switch (which) {
    case 0: return (int)sizeof(sdx_bank_hdr);
    case 1: return (int)sizeof(sdx_patspec);
    case 2: return (int)sizeof(sdx_mu_proto);
    case 3: return (int)sizeof(sdx_ms_proto);
    case 4: return (int)sizeof(sdx_mc_proto);
    case 5: return (int)sizeof(sdx_result);
    case 6: return (int)sizeof(sdx_desc);
    case 7: return (int)sizeof(sdx_mu_desc);
    case 8: return (int)sizeof(sdx_mn_proto);
    case 9: return (int)sizeof(sdx_json_rec);
    case 10: return (int)sizeof(sdx_mu_filt);
    case 11: return (int)sizeof(sdx_ms_filt);
    case 12: return (int)sizeof(sdx_xchg_part);
    case 13: return (int)sizeof(sdx_xchg_wire);
    case 14: return (int)sizeof(sdx_wire_rec);
    case 15: static_assert(sizeof(sdx_msg_rec) == 128, "sdx_msg_rec is one 128-byte line"); return (int)sizeof(sdx_msg_rec);
    case 16: return (int)sizeof(sdx_pulse_batch);
    case 17: return (int)sizeof(sdx_out);
  }
  return -1;
}

int sdx_bank_create(const void* blob, size_t nbytes, int device, sdx_bank** out) {
  if (!blob || !out || nbytes < sizeof(sdx_bank_hdr)) return fail(SDX_EINVAL, "bad bank arguments");
  sdx_bank_hdr h;
  std::memcpy(&h, blob, sizeof h);
  if (h.magic != SDX_BANK_MAGIC || h.version != SDX_BANK_VERSION || h.total_bytes != nbytes)
    return fail(SDX_EBANK, "bank blob magic/version/size mismatch (rebuild the bank and the library)");
  if ((size_t)h.off_order + 2u * ((size_t)h.n_mu + h.n_ms + h.n_mu_groups + 1) > nbytes || h.off_rank > nbytes || h.n_mu > 65535u ||
      h.n_ms > 65535u || (size_t)h.off_mudesc + sizeof(sdx_mu_desc) * h.n_mu > nbytes ||
      (size_t)h.off_mmtab + h.mmtab_bytes > nbytes || h.mmtab_bytes > SDX_MMTAB_LDS || (h.mmtab_bytes & 15u) ||
      (h.off_mudesc & 15u) || (h.off_mmtab & 15u) || 17u * h.mm_states > h.mmtab_bytes || h.n_mn > SDX_MN_MAX ||
      (size_t)h.off_mn + sizeof(sdx_mn_proto) * h.n_mn > nbytes || (h.off_mn & 15u) ||
      (size_t)h.off_json + sizeof(sdx_json_rec) * ((size_t)h.n_mu + h.n_ms + h.n_mc + h.n_mn) > nbytes ||
      (size_t)h.off_mufilt + sizeof(sdx_mu_filt) * h.n_mu > nbytes || (h.off_mufilt & 127u) ||
      (size_t)h.off_msfilt + sizeof(sdx_ms_filt) * h.n_ms > nbytes || (h.off_msfilt & 127u) ||
      (size_t)h.off_mntab + SDX_MNTAB_BYTES > nbytes || (h.off_mntab & 15u))
    return fail(SDX_EBANK, "bank blob: processing-order section out of range");
  HIPCHK(hipSetDevice(device));
  void* d = nullptr;
  HIPCHK(hipMalloc(&d, nbytes));
  hipError_t e = hipMemcpy(d, blob, nbytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return fail(SDX_EHIP, std::string("bank upload: ") + hipGetErrorString(e));
  }
  sdx_bank* b = new sdx_bank{device, d, nbytes, h};
  *out = b;
  return SDX_OK;
}

int sdx_bank_destroy(sdx_bank* bank) {
  if (!bank) return SDX_OK;
  if (bank->dev) (void)hipFree(bank->dev);
  delete bank;
  return SDX_OK;
}

const void* sdx_bank_device_ptr(const sdx_bank* bank) { return bank ? bank->dev : nullptr; }

int sdx_copy_async(void* dst, const void* src, size_t nbytes, void* hip_stream) {
  if (!nbytes) return SDX_OK;
  if (!dst || !src) return fail(SDX_EINVAL, "sdx_copy_async: null pointer");
  HIPCHK(hipMemcpyAsync(dst, src, nbytes, hipMemcpyDefault, (hipStream_t)hip_stream));
  return SDX_OK;
}

int sdx_copy_async_kind(void* dst, const void* src, size_t nbytes, int kind, void* hip_stream) {
  if (!nbytes) return SDX_OK;
  if (!dst || !src) return fail(SDX_EINVAL, "sdx_copy_async_kind: null pointer");
  if (kind < 0 || kind > 4) return fail(SDX_EINVAL, "sdx_copy_async_kind: kind must be a hipMemcpyKind (0-4)");
  HIPCHK(hipMemcpyAsync(dst, src, nbytes, (hipMemcpyKind)kind, (hipStream_t)hip_stream));
  return SDX_OK;
}

int sdx_copy_async_narrow(void* dst, const void* src, size_t nbytes, int nwg, void* hip_stream) {
  if (!nbytes) return SDX_OK;
  if (!dst || !src) return fail(SDX_EINVAL, "sdx_copy_async_narrow: null pointer");
  if (nwg < 1 || nwg > 1024) return fail(SDX_EINVAL, "sdx_copy_async_narrow: 1..1024 workgroups");
  hipLaunchKernelGGL(sdx::k_copy_narrow, dim3(nwg), dim3(256), 0, (hipStream_t)hip_stream, (uint8_t*)dst,
                     (const uint8_t*)src, nbytes);
  HIPCHK(hipGetLastError());
  return SDX_OK;
}

int sdx_fill_async(void* dst, int value, size_t nbytes, void* hip_stream) {
  if (!nbytes) return SDX_OK;
  if (!dst) return fail(SDX_EINVAL, "sdx_fill_async: null pointer");
  HIPCHK(hipMemsetAsync(dst, value, nbytes, (hipStream_t)hip_stream));
  return SDX_OK;
}

int sdx_demod_pulses(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, const sdx_out* out,
                     void* hip_stream) {
  if (!bank || !batch || !out) return fail(SDX_EINVAL, "null argument");
  if (kind != SDX_KIND_MU && kind != SDX_KIND_MS) return fail(SDX_EINVAL, "kind must be MU or MS");
  if (kind == SDX_KIND_MS && (!batch->cp_slot_dev || !batch->ms_ok_dev)) return fail(SDX_EINVAL, "MS needs cp_slot/ms_ok");
  if ((uintptr_t)batch->mrec_dev & 127) return fail(SDX_EINVAL, "mrec_dev must be 128-byte aligned");
  // spill regions are addressed with 32-bit offsets (region index cursor_dev[3] x SPILL_BYTES)
  if (out->work_dev && out->work_cap > 0xFFFFFFFFull - sdx::SPILL_BYTES)
    return fail(SDX_EINVAL, "work_cap above 4 GiB - 112 KB: spill offsets are 32-bit");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  hipStream_t st = (hipStream_t)hip_stream;
  // short variant (<= 256 pulses, 64 messages per tile); the caller routes longer messages (<= 4096)
  // through sel_dev to sdx_demod_pulses_long
  const sdx_pulse_batch& b = *batch;
  const sdx_out& o = *out;
  constexpr int TM = 64;
  const int grid = (ntot + TM - 1) / TM;
  const dim3 blk(sdx::pulses_threads<SDX_KIND_MU, 4>());
  static_assert(sdx::pulses_threads<SDX_KIND_MU, 4>() == sdx::pulses_threads<SDX_KIND_MS, 4>(), "one block shape");
  if (kind == SDX_KIND_MU && b.mrec_dev)
    hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MU, 4, 64, 1>), dim3(grid), blk, 0, st, bank->dev, b, o);
  else if (kind == SDX_KIND_MU)
    hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MU, 4, 64>), dim3(grid), blk, 0, st, bank->dev, b, o);
  else if (b.mrec_dev && SDX_MS_NARROW)
    hipLaunchKernelGGL(sdx::k_ms_classes<1>, dim3(grid), blk, 0, st, bank->dev, b, o);
  else if (b.mrec_dev)
    hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MS, 4, 64, 1>), dim3(grid), blk, 0, st, bank->dev, b, o);
  else if (SDX_MS_NARROW) {
    // MS messages are mostly short (87 % of the bench corpus have <= 128 pulses): tiles whose
    // messages all fit 2 words per id run the NW = 2 instantiation (half the bitmap words and mask
    // arithmetic), the others the NW = 4 one; the grouping puts the long messages last (k_sig)
    static_assert(sdx::pulses_threads<SDX_KIND_MS, 2>() == sdx::pulses_threads<SDX_KIND_MS, 4>(), "block shape");
    // (an NW = 1 class for <= 64 pulses spilled thousands of VGPRs: not used).  One launch decides per
    // tile (k_ms_classes); SDX_MS_TWO_LAUNCHES=1 keeps round 5's two launches over all tiles, each
    // tile returning at once from the other class's launch (A/B)
    if (SDX_MS_TWO_LAUNCHES) {
      hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MS, 2, 64, 0, 1>), dim3(grid), blk, 0, st, bank->dev, b, o);
      hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MS, 4, 64, 0, 3>), dim3(grid), blk, 0, st, bank->dev, b, o);
    } else {
      hipLaunchKernelGGL(sdx::k_ms_classes<0>, dim3(grid), blk, 0, st, bank->dev, b, o);
    }
  } else
    hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MS, 4, 64>), dim3(grid), blk, 0, st, bank->dev, b, o);
  HIPCHK(hipGetLastError());
  return SDX_OK;
}

size_t sdx_pulses_work_bytes(int spill_tiles) { return (size_t)(spill_tiles > 0 ? spill_tiles : 0) * sdx::SPILL_BYTES; }

size_t sdx_group_work_bytes(int n) { return sdx::group_bytes(n); }

int sdx_group_pulses(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, int32_t* order_dev,
                     sdx_msg_rec* mrec_dev, void* work_dev, size_t work_cap, void* hip_stream) {
  if (!bank || !batch || !order_dev || !work_dev) return fail(SDX_EINVAL, "null argument");
  if (kind != SDX_KIND_MU && kind != SDX_KIND_MS) return fail(SDX_EINVAL, "kind must be MU or MS");
  if (kind == SDX_KIND_MS && (!batch->cp_slot_dev || !batch->ms_ok_dev)) return fail(SDX_EINVAL, "MS needs cp_slot/ms_ok");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  if (work_cap < sdx::group_bytes(ntot)) return fail(SDX_EINVAL, "grouping workspace smaller than sdx_group_work_bytes(n)");
  if ((uintptr_t)mrec_dev & 127) return fail(SDX_EINVAL, "mrec_dev must be 128-byte aligned");
  if (!sdx::group_messages(bank->dev, kind, *batch, order_dev, mrec_dev, (uint8_t*)work_dev, work_cap,
                           (hipStream_t)hip_stream))
    return fail(SDX_EHIP, "message grouping (k_sig / radix sort) launch failed");
  return SDX_OK;
}

int sdx_group_step(const sdx_bank* bank, const sdx_group_job* mu, const sdx_group_job* ms, void* hip_stream) {
  if (!bank || !mu || !ms || !mu->batch || !ms->batch) return fail(SDX_EINVAL, "null argument");
  const sdx_group_job* job[2] = {mu, ms};
  for (int k = 0; k < 2; ++k) {
    const sdx_group_job& j = *job[k];
    if (!j.order_dev || !j.work_dev) return fail(SDX_EINVAL, "sdx_group_step: null order / work");
    if ((uintptr_t)j.mrec_dev & 127) return fail(SDX_EINVAL, "mrec_dev must be 128-byte aligned");
    const int n = j.batch->sel_dev ? j.batch->n_sel : j.batch->n;
    if (n > 0 && j.work_cap < sdx::group_bytes(n))
      return fail(SDX_EINVAL, "grouping workspace smaller than sdx_group_work_bytes(n)");
  }
  const int nmu = mu->batch->sel_dev ? mu->batch->n_sel : mu->batch->n;
  const int nms = ms->batch->sel_dev ? ms->batch->n_sel : ms->batch->n;
  if (nms > 0 && (!ms->batch->cp_slot_dev || !ms->batch->ms_ok_dev)) return fail(SDX_EINVAL, "MS needs cp_slot/ms_ok");
  if (nmu <= 0 || nms <= 0) {  // one side empty: the single grouping of the other
    const sdx_group_job& j = nmu > 0 ? *mu : *ms;
    if ((nmu > 0 ? nmu : nms) <= 0) return SDX_OK;
    return sdx_group_pulses(bank, nmu > 0 ? SDX_KIND_MU : SDX_KIND_MS, j.batch, j.order_dev, j.mrec_dev, j.work_dev,
                            j.work_cap, hip_stream);
  }
  if (!sdx::group_messages2(bank->dev, *mu->batch, mu->order_dev, mu->mrec_dev, (uint8_t*)mu->work_dev, mu->work_cap,
                            *ms->batch, ms->order_dev, ms->mrec_dev, (uint8_t*)ms->work_dev, ms->work_cap,
                            (hipStream_t)hip_stream))
    return fail(SDX_EHIP, "message grouping (k_sig2 / radix sort) launch failed");
  return SDX_OK;
}

int sdx_demod_pulses_long(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, const sdx_out* out,
                          void* hip_stream) {
  if (!bank || !batch || !out) return fail(SDX_EINVAL, "null argument");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  hipStream_t st = (hipStream_t)hip_stream;
  constexpr int TM = 4;
  const int grid = (ntot + TM - 1) / TM;
  if (kind == SDX_KIND_MU)
    hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MU, 64, 4>), dim3(grid), dim3(256), 0, st, bank->dev, *batch, *out);
  else if (kind == SDX_KIND_MS)
    hipLaunchKernelGGL((sdx::k_pulses<SDX_KIND_MS, 64, 4>), dim3(grid), dim3(256), 0, st, bank->dev, *batch, *out);
  else
    return fail(SDX_EINVAL, "kind must be MU or MS");
  HIPCHK(hipGetLastError());
  return SDX_OK;
}

static_assert(sdx::MC_SHORTW * 16 == SDX_MC_SHORT_HEX, "k_mc<MC_SHORTW> holds SDX_MC_SHORT_HEX characters");

int sdx_demod_step(const sdx_bank* bank, const sdx_step* step, void* hip_stream) {
  if (!bank || !step) return fail(SDX_EINVAL, "null argument");
  if ((step->mu && !step->mu_out) || (step->ms && !step->ms_out) || (step->mc && !step->mc_out))
    return fail(SDX_EINVAL, "sdx_demod_step: a batch without its sdx_out");
  hipStream_t st = (hipStream_t)hip_stream;
  sdx::StepArgs a{};
  auto count = [](int n, int n_sel, const void* sel) { return sel ? n_sel : n; };
  // the fused kernel's forms: MU short and MS short (the two length classes), each with or without
  // message records, MC frames of <= SDX_MC_SHORT_HEX characters; anything else keeps its own launches,
  // after the fused kernel on the same stream
  const bool ms_fused = step->ms && SDX_MS_NARROW;
  const bool mc_fused = step->mc && step->mc->max_hex > 0 && step->mc->max_hex <= SDX_MC_SHORT_HEX;
  if (step->mc && (int)bank->hdr.n_mc > sdx::MC_CMAXP) return fail(SDX_EINVAL, "the MC kernel's gate mask holds 16 MC protocols");
  if (step->mu) {
    const sdx_pulse_batch& b = *step->mu;
    if ((uintptr_t)b.mrec_dev & 127) return fail(SDX_EINVAL, "mrec_dev must be 128-byte aligned");
    if (step->mu_out->work_dev && step->mu_out->work_cap > 0xFFFFFFFFull - sdx::SPILL_BYTES)
      return fail(SDX_EINVAL, "work_cap above 4 GiB - 112 KB: spill offsets are 32-bit");
    a.mu = b;
    a.mu_out = *step->mu_out;
    a.t_mu = (count(b.n, b.n_sel, b.sel_dev) + 63) / 64;
  }
  if (ms_fused) {
    const sdx_pulse_batch& b = *step->ms;
    if (!b.cp_slot_dev || !b.ms_ok_dev) return fail(SDX_EINVAL, "MS needs cp_slot/ms_ok");
    if ((uintptr_t)b.mrec_dev & 127) return fail(SDX_EINVAL, "mrec_dev must be 128-byte aligned");
    if (step->ms_out->work_dev && step->ms_out->work_cap > 0xFFFFFFFFull - sdx::SPILL_BYTES)
      return fail(SDX_EINVAL, "work_cap above 4 GiB - 112 KB: spill offsets are 32-bit");
    a.ms = b;
    a.ms_out = *step->ms_out;
    a.t_ms = (count(b.n, b.n_sel, b.sel_dev) + 63) / 64;
  }
  if (mc_fused) {
    a.mc = *step->mc;
    a.mc_out = *step->mc_out;
    a.b_mc = (count(a.mc.n, a.mc.n_sel, a.mc.sel_dev) + 511) / 512;
  }
  const long long grid = (long long)a.t_mu + a.t_ms + a.b_mc;
  if (grid > 0x7FFFFFFFll) return fail(SDX_EINVAL, "sdx_demod_step: grid too large");
  if (grid > 0) {
    const bool mru = a.mu.mrec_dev != nullptr, mrs = a.ms.mrec_dev != nullptr;
    if (mru && mrs)
      hipLaunchKernelGGL((sdx::k_step<1, 1>), dim3((unsigned)grid), dim3(512), 0, st, bank->dev, a);
    else if (mru)
      hipLaunchKernelGGL((sdx::k_step<1, 0>), dim3((unsigned)grid), dim3(512), 0, st, bank->dev, a);
    else if (mrs)
      hipLaunchKernelGGL((sdx::k_step<0, 1>), dim3((unsigned)grid), dim3(512), 0, st, bank->dev, a);
    else
      hipLaunchKernelGGL((sdx::k_step<0, 0>), dim3((unsigned)grid), dim3(512), 0, st, bank->dev, a);
    HIPCHK(hipGetLastError());
  }
  if (step->ms && !ms_fused) {
    const int rc = sdx_demod_pulses(bank, SDX_KIND_MS, step->ms, step->ms_out, hip_stream);
    if (rc) return rc;
  }
  if (step->mc && !mc_fused) return sdx_demod_mc(bank, step->mc, step->mc_out, hip_stream);
  return SDX_OK;
}

int sdx_demod_mc(const sdx_bank* bank, const sdx_mc_batch* batch, const sdx_out* out, void* hip_stream) {
  if (!bank || !batch || !out) return fail(SDX_EINVAL, "null argument");
  if ((int)bank->hdr.n_mc > sdx::MC_CMAXP) return fail(SDX_EINVAL, "the MC kernel's gate mask holds 16 MC protocols");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  hipStream_t st = (hipStream_t)hip_stream;
  const int grid = (ntot + 255) / 256;
  hipLaunchKernelGGL((sdx::k_mc<sdx::MC_SHORTW, false>), dim3(grid), dim3(256), 0, st, bank->dev, *batch, *out);
  // the 65..128-character variant only when the caller cannot rule such frames out (VERDICT r04 #4:
  // over a batch without one, its grid of early-exiting waves still held CU slots beside MS)
  if (batch->max_hex <= 0 || batch->max_hex > SDX_MC_SHORT_HEX)
    hipLaunchKernelGGL((sdx::k_mc<sdx::MC_MAXW, true>), dim3(grid), dim3(256), 0, st, bank->dev, *batch, *out);
  HIPCHK(hipGetLastError());
  return SDX_OK;
}

}  // extern "C"
