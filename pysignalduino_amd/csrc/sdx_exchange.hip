// sdx_exchange.hip -- the device side of the multi-GPU exchange (BASELINE config 5).
//
// Every rank demodulates its contiguous shard of the stream; the one exchange step all-gathers the
// decoded dmsg buffers of all ranks over RCCL.  What travels is the wire form of include/sdx.h (v3,
// ABI 11): per launch and rank, in message order, a 4-byte word per message (n_rec, status,
// raise_kind), an 8-byte sdx_wire_rec per record (proto, payload_len, bit_length) and the payloads.
// A payload of the form preamble + uppercase hex digits + postamble of its protocol (the bank's
// affixes: message_unsynced.py:271-274, message_synced.py:228-229, manchester.py:131-132) travels as
// its hex digits packed two per byte (proto bit 15 = SDX_WIRE_NIB); any other payload travels raw.
// rec_begin, payload_off, msg and the affixes are rebuilt by the receiver.
//
// Re-runs: a launch whose messages overflowed (SDX_ST_OVF_TILE / _OUT) is exchanged together with an
// OVERLAY part (sdx_xchg_part.alt): the re-run's outputs, descriptors filled with SDX_ST_ABSENT except
// for the re-run messages.  The sender takes message m from the deepest overlay whose descriptor of m
// is present, so the wire is the same as for a launch that never overflowed.
//
// Sender, two launches around the host's count exchange:
//   k_xw_count  lane = message: resolve the overlay chain, validate the descriptor and its records
//               against the part's cursor / capacities, classify the payloads (raw / nibble), count
//               records, wire payload bytes and payload bytes, block-scan them, block totals;
//   k_xw_scan   one block per launch: exclusive block offsets, the launch's counts;
//   k_xw_words + k_xw_recs (round 6; k_xw_pack before, kept as the SDX_XCHG_PACK_MSG=1 A/B): the wire
//               words (lane = message), then every shipped record with its payload (lane = source
//               record, in each part's own order).  The source records are in tile order (k_pulses
//               places them per tile); the wire is in message order, so the pack is also the
//               canonicalisation that makes sharded and un-sharded runs compare byte for byte.
// Receiver:
//   k_xu_sum / k_xu_scan / k_xu_write / k_xu_heap  rebuild sdx_desc / sdx_result / one contiguous heap
//               of the whole job from the gathered wire sections of every rank.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>

#include "../../include/sdx.h"
#include "../../include/sdx_bank.h"

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
const void* bank_dev_ptr(const sdx_bank* b);
}

namespace sdxx {

constexpr int XT = 256;       // threads per block; one message per thread in the scans
constexpr int XB = XT;        // items per block
constexpr int XMAX = SDX_XCHG_MAX_PARTS;
constexpr int XRANKS = SDX_XCHG_MAX_RANKS;
constexpr uint64_t BADBIT = 1ull << 63;
constexpr int CHAIN = 8;      // overlays per launch (general-path rows, re-runs, re-runs of re-runs)

// Inter-block results travel through kernel boundaries only (count -> scan -> pack): a grid-wide
// "last block" protocol needs agent-scope release fences, and on a multi-XCD part each one writes
// back the whole L2 -- under a concurrently running demodulation kernel that cost ~100 us per launch.

__host__ __device__ inline uint32_t nblk_of(uint64_t n) { return n ? (uint32_t)((n + XB - 1) / XB) : 1u; }
__host__ __device__ inline uint64_t r16(uint64_t x) { return (x + 15) & ~15ull; }
// workspace: a 256-byte head (bad-message counters of parts 0..XMAX-1 at fixed places, so one zeroed
// workspace serves any layout), then per part: loc u64[n] | raw u32[n] | blk u64[nblk] | rawblk u32[nblk]
constexpr uint64_t WHEAD = 256;
__host__ __device__ inline uint64_t part_work_bytes(uint32_t n) {
  return (12ull * n + 12ull * nblk_of(n) + 255) / 256 * 256;
}

struct Parts {
  sdx_xchg_part p[XMAX];
  uint64_t work_off[XMAX];
  int owner[XMAX];      // the launch each part's records ship in (itself, or the launch it overlays); -1 none
  int shared;           // an overlay on the chains of two launches (k_xw_recs assumes one owner per part)
  const uint8_t* bank;  // nullptr: raw payloads only
  int k;
};

struct PartWork {
  uint32_t* bad;   // bad messages (reset by k_xw_scan)
  uint64_t* loc;   // per message: BADBIT | local record prefix << 32 | local wire byte prefix (in its block)
  uint32_t* raw;   // per message: local payload byte prefix
  uint64_t* blk;   // block totals -> exclusive block offsets (records << 32 | wire bytes)
  uint32_t* rawblk;
};

__device__ inline PartWork part_work(uint8_t* work, const Parts& P, int k) {
  PartWork w;
  const uint32_t n = P.p[k].n_msgs;
  uint8_t* b = work + WHEAD + P.work_off[k];
  w.bad = reinterpret_cast<uint32_t*>(work) + k;
  w.loc = reinterpret_cast<uint64_t*>(b);
  w.blk = w.loc + n;
  w.raw = reinterpret_cast<uint32_t*>(w.blk + nblk_of(n));
  w.rawblk = w.raw + n;
  return w;
}

__device__ inline int lane_id() { return (int)__lane_id(); }

// (records << 32 | bytes) pairs: the low halves sum payload bytes of one launch (< 2^32, the heap is
// u32-addressed), the high halves records, so a 64-bit add never carries between them.
__device__ inline uint64_t wave_incl(uint64_t v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(v, o);
    if (lane_id() >= o) v += y;
  }
  return v;
}

// exclusive block scan of one u64 per thread; *total = the block's sum
__device__ inline uint64_t block_excl(uint64_t v, uint64_t* total) {
  __shared__ uint64_t wsum[XT / 64];
  const uint64_t inc = wave_incl(v);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 63) wsum[w] = inc;
  __syncthreads();
  uint64_t base = 0, all = 0;
#pragma unroll
  for (int i = 0; i < XT / 64; ++i) {
    const uint64_t s = wsum[i];
    base += i < w ? s : 0;
    all += s;
  }
  __syncthreads();  // wsum is reused by the next call
  *total = all;
  return base + inc - v;
}

// in-place exclusive scan of blk[0, nb) by one block; returns the sum
__device__ inline uint64_t block_scan_array(uint64_t* blk, uint32_t nb) {
  uint64_t carry = 0;
  for (uint32_t c = 0; c < nb; c += XT) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < nb ? blk[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl(v, &tot);
    if (i < nb) blk[i] = carry + ex;
    carry += tot;
  }
  return carry;
}
__device__ inline uint32_t block_scan_array32(uint32_t* blk, uint32_t nb) {
  uint64_t carry = 0;
  for (uint32_t c = 0; c < nb; c += XT) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < nb ? blk[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl(v, &tot);
    if (i < nb) blk[i] = (uint32_t)(carry + ex);
    carry += tot;
  }
  return (uint32_t)carry;
}

// ---- payload affixes and the nibble form ----------------------------------------------------------
struct Affix {
  const uint8_t* pre;
  const uint8_t* post;
  uint32_t npre, npost;
  bool ok;  // the bank knows the protocol: the nibble form applies
};

__device__ inline Affix affix_of(const uint8_t* bank, int kind, uint32_t proto) {
  Affix a{nullptr, nullptr, 0, 0, false};
  if (!bank) return a;
  const sdx_bank_hdr* h = reinterpret_cast<const sdx_bank_hdr*>(bank);
  const uint8_t* str = bank + h->off_str;
  int32_t po = 0, pl = 0, qo = 0, ql = 0;
  if (kind == SDX_KIND_MU && proto < h->n_mu) {
    const sdx_mu_proto& p = reinterpret_cast<const sdx_mu_proto*>(bank + h->off_mu)[proto];
    po = p.pre_off, pl = p.pre_len, qo = p.post_off, ql = p.post_len;
  } else if (kind == SDX_KIND_MS && proto < h->n_ms) {
    const sdx_ms_proto& p = reinterpret_cast<const sdx_ms_proto*>(bank + h->off_ms)[proto];
    po = p.pre_off, pl = p.pre_len, qo = p.post_off, ql = p.post_len;
  } else if (kind == SDX_KIND_MC && proto < h->n_mc) {
    const sdx_mc_proto& p = reinterpret_cast<const sdx_mc_proto*>(bank + h->off_mc)[proto];
    po = p.pre_off, pl = p.pre_len;
  } else if (kind == SDX_KIND_MN && proto < h->n_mn) {
    const sdx_mn_proto& p = reinterpret_cast<const sdx_mn_proto*>(bank + h->off_mn)[proto];
    po = p.pre_off, pl = p.pre_len;
  } else {
    return a;
  }
  a.pre = str + po;
  a.post = str + qo;
  a.npre = (uint32_t)pl;
  a.npost = (uint32_t)ql;
  a.ok = pl >= 0 && ql >= 0;
  return a;
}

__device__ inline bool is_uhex(uint8_t c) { return (uint8_t)(c - '0') < 10u || (uint8_t)(c - 'A') < 6u; }
__device__ inline uint32_t hexval(uint8_t c) { return c <= '9' ? (uint32_t)(c - '0') : (uint32_t)(c - 'A' + 10); }

// payload p[0, len) == pre + D uppercase hex digits + post?  Returns D, or -1 (raw form)
__device__ inline int nib_digits(const Affix& a, const uint8_t* p, uint32_t len) {
  if (!a.ok || a.npre > 255u || len < a.npre + a.npost) return -1;   // npre > 255: raw (as the xrec word)
  for (uint32_t i = 0; i < a.npre; ++i)
    if (p[i] != a.pre[i]) return -1;
  const uint32_t d = len - a.npre - a.npost;
  for (uint32_t i = 0; i < a.npost; ++i)
    if (p[a.npre + d + i] != a.post[i]) return -1;
  for (uint32_t i = 0; i < d; ++i)
    if (!is_uhex(p[a.npre + i])) return -1;
  return (int)d;
}

__device__ inline uint32_t wire_bytes_of(int digits, uint32_t len) {
  return digits >= 0 ? ((uint32_t)digits + 1) >> 1 : len;
}

// the nibble form applies to a part's payloads at all (a bank and the part's protocol kind)
__device__ inline bool nibble_on(const Parts& P, const sdx_xchg_part& x) {
  return P.bank != nullptr && x.kind <= SDX_KIND_MN;
}

// ---- sender ---------------------------------------------------------------------------------------
__device__ inline void clamp_counts(const sdx_xchg_part& x, uint32_t* nrec_c, uint32_t* nheap_c) {
  const uint32_t c0 = x.cursor_dev[0], c1 = x.cursor_dev[1];
  *nrec_c = c0 < x.rec_cap ? c0 : x.rec_cap;
  *nheap_c = c1 < x.heap_cap ? c1 : x.heap_cap;
}

// message m of part k: the LAST overlay along the chain k -> alt -> alt ... whose descriptor of m is
// present (later overlays take precedence: e.g. general-path rows, then the re-runs of overflows)
__device__ inline int resolve(const Parts& P, int k, uint32_t m, sdx_desc* d) {
  *d = reinterpret_cast<const sdx_desc*>(P.p[k].desc_dev)[m];
  int res = k, c = k;
  for (int hop = 0; hop < CHAIN; ++hop) {
    const int a = (int)P.p[c].alt - 1;
    if (a < 0 || a >= P.k) break;
    const sdx_desc da = reinterpret_cast<const sdx_desc*>(P.p[a].desc_dev)[m];
    if (da.status != SDX_ST_ABSENT) {
      res = a;
      *d = da;
    }
    c = a;
  }
  return res;
}

// the validated (records << 32 | wire payload bytes) of message m and its payload bytes; *ok = false
// marks a message the exchange cannot ship (an overflow status, or a descriptor / record outside
// what the launch wrote)
__device__ inline uint64_t msg_counts(const Parts& P, int k0, uint32_t m, bool* ok, uint32_t* rawb) {
  sdx_desc d;
  const int k = resolve(P, k0, m, &d);
  const sdx_xchg_part& x = P.p[k];
  *ok = true;
  *rawb = 0;
  if (d.status == SDX_ST_RAISED) return 0;
  uint32_t nrec_c, nheap_c;
  clamp_counts(x, &nrec_c, &nheap_c);
  if (d.status != SDX_ST_OK || (d.n_rec && (uint64_t)d.rec_begin + d.n_rec > nrec_c)) {
    *ok = false;
    return 0;
  }
  if (x.wire_dev) {  // ABI 12: the launch's kernel counted the message while its payloads were on chip
    const uint64_t w = x.wire_dev[m];
    const uint32_t rb = (uint32_t)(w >> 32);
    *rawb = rb;
    return ((uint64_t)d.n_rec << 32) | (nibble_on(P, x) ? (uint32_t)w : rb);
  }
  const sdx_result* r = reinterpret_cast<const sdx_result*>(x.rec_dev) + d.rec_begin;
  uint64_t bytes = 0, raw = 0;
  bool good = true;
  for (uint32_t j = 0; j < d.n_rec; ++j) {
    const sdx_result v = r[j];
    const bool in = v.msg == m && (uint64_t)v.payload_off + v.payload_len <= nheap_c;
    good &= in;
    if (!in) continue;
    const int dg = nib_digits(affix_of(P.bank, x.kind, v.proto), x.heap_dev + v.payload_off, v.payload_len);
    bytes += wire_bytes_of(dg, v.payload_len);
    raw += v.payload_len;
  }
  *ok = good;
  *rawb = good ? (uint32_t)raw : 0u;
  return good ? (((uint64_t)d.n_rec << 32) | bytes) : 0;
}

// lane = message: validate, count, block-local prefixes; block totals for k_xw_scan
__global__ __launch_bounds__(XT) void k_xw_count(Parts P, uint8_t* __restrict__ work) {
  const int k = blockIdx.y;
  const sdx_xchg_part& x = P.p[k];
  if (x.aux || blockIdx.x >= nblk_of(x.n_msgs)) return;
  PartWork w = part_work(work, P, k);
  const uint32_t m = blockIdx.x * XB + threadIdx.x;
  bool ok = true;
  uint32_t rawb = 0;
  const uint64_t v = m < x.n_msgs ? msg_counts(P, k, m, &ok, &rawb) : 0;
  uint64_t tot, rtot;
  const uint64_t pre = block_excl(v, &tot);
  const uint64_t rpre = block_excl(rawb, &rtot);
  if (m < x.n_msgs) {
    w.loc[m] = pre | (ok ? 0 : BADBIT);
    w.raw[m] = (uint32_t)rpre;
  }
  const uint64_t bad_wave = __ballot(!ok);
  if (lane_id() == 0 && bad_wave) atomicAdd(w.bad, (uint32_t)__popcll(bad_wave));
  if (threadIdx.x == 0) {
    w.blk[blockIdx.x] = tot;
    w.rawblk[blockIdx.x] = (uint32_t)rtot;
  }
}

// one block per launch: block offsets, the launch's counts
__global__ __launch_bounds__(XT) void k_xw_scan(Parts P, uint8_t* __restrict__ work, uint32_t* __restrict__ counts) {
  const int k = blockIdx.x;
  const sdx_xchg_part& x = P.p[k];
  uint32_t* c = counts + SDX_XCHG_COUNTS * k;
  if (x.aux) {  // an overlay: its messages travel in the part it overlays
    if (threadIdx.x < SDX_XCHG_COUNTS) c[threadIdx.x] = 0;
    return;
  }
  PartWork w = part_work(work, P, k);
  const uint64_t all = block_scan_array(w.blk, nblk_of(x.n_msgs));
  const uint32_t rall = block_scan_array32(w.rawblk, nblk_of(x.n_msgs));
  if (threadIdx.x == 0) {
    c[0] = x.n_msgs;
    c[1] = (uint32_t)(all >> 32);
    c[2] = (uint32_t)all;
    c[3] = *w.bad;
    c[4] = rall;
    c[5] = c[6] = c[7] = 0;
    *w.bad = 0;
  }
}

// the send layout, in launch order: [msg | rec | heap] sections of each launch, 16-byte aligned
__device__ inline void section_offsets(const uint32_t* counts, int K, int k, uint64_t* o) {
  uint64_t off = 0;
  for (int i = 0; i < K; ++i) {
    const uint32_t* c = counts + SDX_XCHG_COUNTS * i;
    if (i == k) {
      o[0] = off;
      o[1] = off + r16(4ull * c[0]);
      o[2] = o[1] + r16(8ull * c[1]);
      return;
    }
    off += r16(4ull * c[0]) + r16(8ull * c[1]) + r16(c[2]);
  }
}

__device__ inline void zero_tail(uint8_t* sec, uint64_t used, uint32_t lane) {
  if (lane < 16 && used + lane < r16(used)) sec[used + lane] = 0;
}

// the bytes [p, p + n) (n <= 8) of a payload as a little-endian word: aligned dword loads, only of
// dwords that hold one of those bytes (each lies inside the payload's allocation), realigned
__device__ inline uint64_t load_le(const uint8_t* p, uint32_t n) {
  const uint32_t sh = (uint32_t)(uintptr_t)p & 3u;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(p - sh);
  const uint32_t w0 = a[0];
  const uint32_t w1 = sh + n > 4 ? a[1] : 0u;
  const uint32_t w2 = sh + n > 8 ? a[2] : 0u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  const uint64_t x = ((uint64_t)hi << 32) | lo;
  return n >= 8 ? x : x & ((1ull << (8 * n)) - 1);
}

// one record's wire bytes: dg < 0 copies its n payload bytes; dg >= 0 packs its dg uppercase hex
// digits two per byte (high nibble first; an odd last digit in a high nibble), n = (dg + 1) / 2
__device__ inline void wire_copy(uint8_t* dst, const uint8_t* src, int dg, uint32_t n) {
  for (uint32_t q = 0; q < n; q += 4) {
    const uint32_t cnt = n - q < 4 ? n - q : 4;
    uint32_t out;
    if (dg < 0) {
      out = (uint32_t)load_le(src + q, cnt);
    } else {
      const uint32_t nd = (uint32_t)dg - 2 * q < 8 ? (uint32_t)dg - 2 * q : 8;   // digits of this step (>= 1)
      const uint64_t x = load_le(src + 2 * q, nd);
      // '0'-'9' -> 0-9, 'A'-'F' -> 10-15 (bit 6 set); the bytes past the digits are zero
      const uint64_t v = (x & 0x0F0F0F0F0F0F0F0Full) + 9ull * ((x >> 6) & 0x0101010101010101ull);
      uint64_t y = ((v & 0x00FF00FF00FF00FFull) << 4) | ((v >> 8) & 0x00FF00FF00FF00FFull);  // digit pairs
      y = (y | (y >> 8)) & 0x0000FFFF0000FFFFull;
      out = (uint32_t)(y | (y >> 16));
    }
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if ((uint32_t)b < cnt) dst[q + b] = (uint8_t)(out >> (8 * b));
  }
}

// block = 256 consecutive messages (the count blocks), grid.y = launch.
// A (lane = message): the wire word; the message's first record (block-local record prefix of the
//   count), its resolved part and rec_begin into LDS;
// B (lane = record, chunks of 256 in output order): the record's message by a binary search over the
//   record prefixes, its sdx_result and class (the kernel-written xrec, or the scan), the wire record,
//   a block scan of the wire bytes for its destination, and its payload bytes (wire_copy).
// Every lane has work in both phases (round 3's phase A looped over each message's records with the
// other lanes idle, and its payload phase took one lane per 32 output bytes: 182 VGPRs, 2 waves/SIMD,
// 200 us for the bench step's 1M messages in the nibble form).
__global__ __launch_bounds__(XT) void k_xw_pack(Parts P, const uint32_t* __restrict__ counts,
                                                uint8_t* __restrict__ work, uint8_t* __restrict__ send) {
  __shared__ uint32_t l_r0[XB + 1];  // block-local index of each message's first record (+ the end)
  __shared__ uint32_t l_rb[XB];      // its rec_begin in the resolved part
  __shared__ uint8_t l_pt[XB];       // the resolved part
  const int k = blockIdx.y;
  const sdx_xchg_part& x = P.p[k];
  const uint32_t nb = nblk_of(x.n_msgs);
  if (x.aux || blockIdx.x >= nb) return;
  PartWork w = part_work(work, P, k);
  const uint32_t* ck = counts + SDX_XCHG_COUNTS * k;
  uint64_t so[3];
  section_offsets(counts, P.k, k, so);
  uint8_t* s_msg = send + so[0];
  sdx_wire_rec* s_rec = reinterpret_cast<sdx_wire_rec*>(send + so[1]);
  uint8_t* s_heap = send + so[2];
  if (blockIdx.x == 0) {  // deterministic section padding
    zero_tail(s_msg, 4ull * x.n_msgs, threadIdx.x);
    zero_tail(reinterpret_cast<uint8_t*>(s_rec), 8ull * ck[1], threadIdx.x);
    zero_tail(s_heap, ck[2], threadIdx.x);
  }
  const uint64_t boff = w.blk[blockIdx.x];
  const uint64_t bnext = blockIdx.x + 1 < nb ? w.blk[blockIdx.x + 1] : (((uint64_t)ck[1] << 32) | ck[2]);
  const uint32_t brec = (uint32_t)((bnext >> 32) - (boff >> 32));   // the block's records
  const uint32_t tid = threadIdx.x;
  const uint32_t m = blockIdx.x * XB + tid;
  if (m < x.n_msgs) {
    sdx_desc d;
    const int kr = resolve(P, k, m, &d);
    const uint64_t loc = w.loc[m];
    const bool bad = (loc & BADBIT) != 0;
    const uint32_t nr = (bad || d.status != SDX_ST_OK) ? 0u : d.n_rec;
    reinterpret_cast<uint32_t*>(s_msg)[m] =
        nr | ((uint32_t)(bad ? SDX_ST_OVF_OUT : d.status) << 16) | ((uint32_t)d.raise_kind << 24);
    l_r0[tid] = (uint32_t)((loc & ~BADBIT) >> 32);
    l_rb[tid] = d.rec_begin;
    l_pt[tid] = (uint8_t)kr;
  } else {
    l_r0[tid] = brec;   // past the launch's messages: no records
  }
  if (tid == 0) l_r0[XB] = brec;
  __syncthreads();
  uint8_t* bh = s_heap + (uint32_t)boff;
  uint32_t carry = 0;   // block-local wire byte offset of the chunk
  for (uint32_t c = 0; c < brec; c += XT) {   // block-uniform trip count (the scan below)
    const uint32_t r = c + tid;
    uint32_t wl = 0;
    int dg = -1;
    const uint8_t* s0 = nullptr;
    if (r < brec) {
      uint32_t lo = 0, hi = XB - 1;   // the last message whose first record is <= r
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (l_r0[mid] <= r) lo = mid;
        else hi = mid - 1;
      }
      const sdx_xchg_part& y = P.p[l_pt[lo]];
      const uint32_t ri = l_rb[lo] + (r - l_r0[lo]);
      const sdx_result rr = reinterpret_cast<const sdx_result*>(y.rec_dev)[ri];
      const uint8_t* src = y.heap_dev + rr.payload_off;
      uint32_t npre = 0;
      if (y.xrec_dev) {  // ABI 12: classified by the launch's kernel
        const uint32_t xr = nibble_on(P, y) ? y.xrec_dev[ri] : 0u;
        dg = (xr & SDX_XREC_NIB) ? (int)(xr & 0xFFFFu) : -1;
        npre = (xr >> 16) & 0xFFu;
      } else {
        const Affix a = affix_of(P.bank, y.kind, rr.proto);
        dg = nib_digits(a, src, rr.payload_len);
        npre = a.npre;
      }
      sdx_wire_rec o;
      o.proto = (uint16_t)(rr.proto | (dg >= 0 ? SDX_WIRE_NIB : 0u));
      o.payload_len = rr.payload_len;
      o.bit_length = rr.bit_length;
      s_rec[(uint32_t)(boff >> 32) + r] = o;
      s0 = dg >= 0 ? src + npre : src;
      wl = wire_bytes_of(dg, rr.payload_len);
    }
    uint64_t tot;
    const uint32_t pre = (uint32_t)block_excl(wl, &tot);
    if (wl) wire_copy(bh + carry + pre, s0, dg, wl);
    carry += (uint32_t)tot;
  }
}

// ---- the pack in source-record order (round 6) -----------------------------------------------------
// k_xw_pack reads the launches' records in WIRE order (message order): the grouping puts consecutive
// messages in different tiles, so every message's records and payloads are a dependent, scattered
// read (desc -> record -> payload), and under a concurrently running k_step those latencies are what
// the pack costs.  The same bytes are produced here from the other side:
//   k_xw_words  lane = message: the wire word (coalesced descriptor reads);
//   k_xw_recs   lane = source record of a part (primary or overlay), in the part's own order, so the
//               record, xrec and payload reads stream; the record's message (sdx_result.msg) gives its
//               wire place: the message's record / wire-byte prefix from the count (loc + blk) plus its
//               index in the message and the wire bytes of the message's earlier records (a wave scan;
//               a message that began in an earlier wave adds them by a short loop).  A record is
//               shipped iff its message resolves to this part, is shippable (not bad, status OK) and its
//               range holds the record -- exactly the records the count counted, each once.
// The stores are scattered instead (fire-and-forget, runs of ~4 records per message).
__global__ __launch_bounds__(XT) void k_xw_words(Parts P, const uint32_t* __restrict__ counts,
                                                 uint8_t* __restrict__ work, uint8_t* __restrict__ send) {
  const int k = blockIdx.y;
  const sdx_xchg_part& x = P.p[k];
  if (x.aux || blockIdx.x >= nblk_of(x.n_msgs)) return;
  PartWork w = part_work(work, P, k);
  const uint32_t* ck = counts + SDX_XCHG_COUNTS * k;
  uint64_t so[3];
  section_offsets(counts, P.k, k, so);
  uint8_t* s_msg = send + so[0];
  if (blockIdx.x == 0) {  // deterministic section padding
    zero_tail(s_msg, 4ull * x.n_msgs, threadIdx.x);
    zero_tail(send + so[1], 8ull * ck[1], threadIdx.x);
    zero_tail(send + so[2], ck[2], threadIdx.x);
  }
  const uint32_t m = blockIdx.x * XB + threadIdx.x;
  if (m < x.n_msgs) {
    sdx_desc d;
    resolve(P, k, m, &d);
    const bool bad = (w.loc[m] & BADBIT) != 0;
    const uint32_t nr = (bad || d.status != SDX_ST_OK) ? 0u : d.n_rec;
    reinterpret_cast<uint32_t*>(s_msg)[m] =
        nr | ((uint32_t)(bad ? SDX_ST_OVF_OUT : d.status) << 16) | ((uint32_t)d.raise_kind << 24);
  }
}

// the wire bytes of record t of part y (its class as the pack below decides it)
__device__ inline uint32_t rec_wire_bytes(const Parts& P, const sdx_xchg_part& y, uint32_t t) {
  const sdx_result rr = reinterpret_cast<const sdx_result*>(y.rec_dev)[t];
  int dg;
  if (y.xrec_dev) {
    const uint32_t xr = nibble_on(P, y) ? y.xrec_dev[t] : 0u;
    dg = (xr & SDX_XREC_NIB) ? (int)(xr & 0xFFFFu) : -1;
  } else {
    dg = nib_digits(affix_of(P.bank, y.kind, rr.proto), y.heap_dev + rr.payload_off, rr.payload_len);
  }
  return wire_bytes_of(dg, rr.payload_len);
}

// grid (record blocks, parts): blockIdx.y = the source part y, owner[y] = the launch it ships in
constexpr uint32_t XREC_GRID = 1u << 20;  // record blocks per part: one per 256 records of the capacity
__global__ __launch_bounds__(XT) void k_xw_recs(Parts P, const uint32_t* __restrict__ counts,
                                                uint8_t* __restrict__ work, uint8_t* __restrict__ send) {
  const int y = blockIdx.y;
  const sdx_xchg_part& yp = P.p[y];
  const int k = P.owner[y];
  if (k < 0) return;
  uint32_t nrec_c, nheap_c;
  clamp_counts(yp, &nrec_c, &nheap_c);
  if (blockIdx.x * XB >= nrec_c) return;  // block-uniform
  const sdx_xchg_part& x = P.p[k];
  PartWork w = part_work(work, P, k);
  uint64_t so[3];
  section_offsets(counts, P.k, k, so);
  sdx_wire_rec* s_rec = reinterpret_cast<sdx_wire_rec*>(send + so[1]);
  uint8_t* s_heap = send + so[2];
  const int lane = lane_id();
  // grid-stride over the part's records: the grid is sized from the capacities (the cursor is on the
  // device), so a fixed number of blocks walks [0, cursor) instead of one block per capacity chunk
  for (uint32_t c0 = blockIdx.x * XB; c0 < nrec_c; c0 += gridDim.x * XB) {
  const uint32_t i = c0 + threadIdx.x;
  bool ok = false;
  uint32_t m = 0, j = 0, rb = 0, wl = 0;
  int dg = -1;
  const uint8_t* s0 = nullptr;
  uint64_t dst_rec = 0, dst_msg = 0;  // the message's first wire record / its wire payload offset
  uint32_t nr = 0, tot_m = 0;         // the message's records and wire payload bytes
  if (i < nrec_c) {
    const sdx_result rr = reinterpret_cast<const sdx_result*>(yp.rec_dev)[i];
    m = rr.msg;
    if (m < x.n_msgs) {
      sdx_desc d;
      const int kr = resolve(P, k, m, &d);
      const uint64_t loc = w.loc[m];
      ok = kr == y && d.status == SDX_ST_OK && !(loc & BADBIT) && i >= d.rec_begin && i - d.rec_begin < d.n_rec;
      if (ok) {
        rb = d.rec_begin;
        j = i - d.rec_begin;
        const uint64_t b = w.blk[m / XB];
        dst_rec = (b >> 32) + (loc >> 32);
        dst_msg = (uint32_t)b + (uint32_t)loc;
        nr = d.n_rec;
        const uint32_t m1 = m + 1;  // the next message's wire payload offset (the launch's total at the end)
        const uint32_t wend = m1 < x.n_msgs ? (uint32_t)w.blk[m1 / XB] + (uint32_t)w.loc[m1]
                                            : counts[SDX_XCHG_COUNTS * k + 2];
        tot_m = wend - (uint32_t)dst_msg;
        const uint8_t* src = yp.heap_dev + rr.payload_off;
        uint32_t npre = 0;
        if (yp.xrec_dev) {
          const uint32_t xr = nibble_on(P, yp) ? yp.xrec_dev[i] : 0u;
          dg = (xr & SDX_XREC_NIB) ? (int)(xr & 0xFFFFu) : -1;
          npre = (xr >> 16) & 0xFFu;
        } else {
          const Affix a = affix_of(P.bank, yp.kind, rr.proto);
          dg = nib_digits(a, src, rr.payload_len);
          npre = a.npre;
        }
        sdx_wire_rec o;
        o.proto = (uint16_t)(rr.proto | (dg >= 0 ? SDX_WIRE_NIB : 0u));
        o.payload_len = rr.payload_len;
        o.bit_length = rr.bit_length;
        s_rec[dst_rec + j] = o;
        s0 = dg >= 0 ? src + npre : src;
        wl = wire_bytes_of(dg, rr.payload_len);
      }
    }
  }
  // the wire bytes of the message's records before this one, from the wave's scan: counted forward
  // from the message's first lane when it starts in this wave; otherwise backward from its total
  // (the count's prefixes) when it ends in this wave; a message spanning the whole wave (more than 64
  // records, rare) has lane 0 add up its earlier records
  uint32_t inc = wl;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  const uint32_t exc = inc - wl;
  const int head = ok ? lane - (int)j : lane;            // the message's first lane (< 0: an earlier wave)
  const int tail = ok ? lane + (int)(nr - 1 - j) : lane;  // its last lane (> 63: a later wave)
  const uint32_t at_head = __shfl(exc, head > 0 ? head : 0);
  const uint32_t at_tail = __shfl(inc, tail < 63 ? tail : 63);
  uint32_t carry = 0;
  if (lane == 0 && ok && j > 0 && tail > 63) {
    for (uint32_t t = rb; t < i; ++t) carry += rec_wire_bytes(P, yp, t);
  }
  carry = __shfl(carry, 0);
  if (ok && wl) {
    const uint32_t pre = head >= 0 ? exc - at_head : (tail <= 63 ? tot_m - (at_tail - exc) : exc + carry);
    wire_copy(s_heap + dst_msg + pre, s0, dg, wl);
  }
  }
}

// ---- receiver ------------------------------------------------------------------------------------
struct Wire {
  sdx_xchg_wire r[XRANKS];
  uint32_t msg0[XRANKS + 1];   // first global message of rank r
  uint32_t rec0[XRANKS + 1];   // first global record
  uint32_t wire0[XRANKS + 1];  // first global wire payload byte
  const uint8_t* bank;
  int nranks, kind;
};

__device__ inline int rank_of(const uint32_t* start, int nr, uint32_t g) {
  int lo = 0, hi = nr - 1;  // the last r with start[r] <= g
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (start[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ inline sdx_wire_rec wrec_at(const Wire& W, uint32_t g) {
  const int r = rank_of(W.rec0, W.nranks, g);
  return reinterpret_cast<const sdx_wire_rec*>(W.r[r].rec_dev)[g - W.rec0[r]];
}

// digits of a nibble-form record (its payload minus the affixes)
__device__ inline uint32_t wire_len(const Wire& W, const sdx_wire_rec& wr) {
  if (!(wr.proto & SDX_WIRE_NIB)) return wr.payload_len;
  const Affix a = affix_of(W.bank, W.kind, wr.proto & (SDX_WIRE_NIB - 1u));
  const uint32_t dg = wr.payload_len - a.npre - a.npost;
  return (dg + 1) >> 1;
}

// items: global messages [0, M) (value: records << 32) in blocks [0, nbm), global records [0, R)
// (value: payload bytes << 32 | wire bytes) in blocks [nbm, nbm + nbr)
__device__ inline uint64_t xu_item(const Wire& W, bool is_msg, uint32_t g, uint32_t M, uint32_t R) {
  if (is_msg) {
    if (g >= M) return 0;
    const int r = rank_of(W.msg0, W.nranks, g);
    const uint32_t word = reinterpret_cast<const uint32_t*>(W.r[r].msg_dev)[g - W.msg0[r]];
    return (uint64_t)(word & 0xffffu) << 32;
  }
  if (g >= R) return 0;
  const sdx_wire_rec wr = wrec_at(W, g);
  return ((uint64_t)wr.payload_len << 32) | wire_len(W, wr);
}

__global__ __launch_bounds__(XT) void k_xu_sum(Wire W, uint8_t* __restrict__ work) {
  const uint32_t M = W.msg0[W.nranks], R = W.rec0[W.nranks];
  const uint32_t nbm = nblk_of(M);
  uint64_t* blk = reinterpret_cast<uint64_t*>(work + 64);
  const bool is_msg = blockIdx.x < nbm;
  const uint32_t b = is_msg ? blockIdx.x : blockIdx.x - nbm;
  uint64_t tot;
  (void)block_excl(xu_item(W, is_msg, b * XB + threadIdx.x, M, R), &tot);
  if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

__global__ __launch_bounds__(XT) void k_xu_scan(Wire W, uint8_t* __restrict__ work) {
  const uint32_t M = W.msg0[W.nranks], R = W.rec0[W.nranks];
  const uint32_t nbm = nblk_of(M), nbr = nblk_of(R);
  uint64_t* blk = reinterpret_cast<uint64_t*>(work + 64);
  block_scan_array(blk, nbm);
  const uint64_t all = block_scan_array(blk + nbm, nbr);
  if (threadIdx.x == 0) reinterpret_cast<uint64_t*>(work)[0] = all;   // payload bytes << 32 | wire bytes
}

// blocks [0, nbm): descriptors (and each record's msg field); [nbm, nbm + nbr): records (and the
// record's global wire byte offset into the workspace, for k_xu_heap)
__global__ __launch_bounds__(XT) void k_xu_write(Wire W, uint8_t* __restrict__ work, sdx_desc* __restrict__ desc,
                                                 sdx_result* __restrict__ rec) {
  const uint32_t M = W.msg0[W.nranks], R = W.rec0[W.nranks];
  const uint32_t nbm = nblk_of(M), nbr = nblk_of(R);
  const uint64_t* blk = reinterpret_cast<const uint64_t*>(work + 64);
  uint32_t* wsrc = reinterpret_cast<uint32_t*>(work + 64 + 8ull * (nbm + nbr));
  const bool is_msg = blockIdx.x < nbm;
  const uint32_t g = (is_msg ? blockIdx.x : blockIdx.x - nbm) * XB + threadIdx.x;
  const uint64_t v = xu_item(W, is_msg, g, M, R);
  uint64_t tot;
  const uint64_t pre = block_excl(v, &tot) + blk[blockIdx.x];
  if (is_msg && g < M) {
    const int r = rank_of(W.msg0, W.nranks, g);
    const uint32_t word = reinterpret_cast<const uint32_t*>(W.r[r].msg_dev)[g - W.msg0[r]];
    sdx_desc o;
    o.rec_begin = (uint32_t)(pre >> 32);
    o.n_rec = (uint16_t)(word & 0xffffu);
    o.status = (uint8_t)(word >> 16);
    o.raise_kind = (uint8_t)(word >> 24);
    desc[g] = o;
    for (uint32_t i = 0; i < o.n_rec; ++i) rec[o.rec_begin + i].msg = g;
  } else if (!is_msg && g < R) {
    const sdx_wire_rec wr = wrec_at(W, g);
    sdx_result* o = rec + g;
    o->payload_off = (uint32_t)(pre >> 32);
    o->payload_len = wr.payload_len;
    o->proto = (uint16_t)(wr.proto & (SDX_WIRE_NIB - 1u));
    o->bit_length = wr.bit_length;
    wsrc[g] = (uint32_t)pre | ((wr.proto & SDX_WIRE_NIB) ? 0x80000000u : 0u);
  }
}

// lane = record: its payload into the heap (raw copy, or preamble + the digits + postamble)
__global__ __launch_bounds__(XT) void k_xu_heap(Wire W, const uint8_t* __restrict__ work,
                                                const sdx_result* __restrict__ rec, uint8_t* __restrict__ heap) {
  const uint32_t M = W.msg0[W.nranks], R = W.rec0[W.nranks];
  const uint32_t nbm = nblk_of(M), nbr = nblk_of(R);
  const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(work + 64 + 8ull * (nbm + nbr));
  const uint32_t g = blockIdx.x * XT + threadIdx.x;
  if (g >= R) return;
  const sdx_result o = rec[g];
  const uint32_t ws = wsrc[g] & 0x7fffffffu;
  const bool nib = (wsrc[g] & 0x80000000u) != 0;
  const int r = rank_of(W.wire0, W.nranks, ws);
  const uint8_t* src = W.r[r].heap_dev + (ws - W.wire0[r]);
  uint8_t* dst = heap + o.payload_off;
  if (!nib) {
    for (uint32_t i = 0; i < o.payload_len; ++i) dst[i] = src[i];
    return;
  }
  const Affix a = affix_of(W.bank, W.kind, o.proto);
  const uint32_t dg = o.payload_len - a.npre - a.npost;
  for (uint32_t i = 0; i < a.npre; ++i) dst[i] = a.pre[i];
  for (uint32_t i = 0; i < dg; ++i) {
    const uint32_t v = (src[i >> 1] >> ((i & 1) ? 0 : 4)) & 15u;
    dst[a.npre + i] = (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10);
  }
  for (uint32_t i = 0; i < a.npost; ++i) dst[a.npre + dg + i] = a.post[i];
}

}  // namespace sdxx

using namespace sdxx;

extern "C" uint64_t sdx_exchange_work_bytes(const uint32_t* n_msgs, int k) {
  uint64_t s = WHEAD;
  for (int i = 0; i < k; ++i) s += part_work_bytes(n_msgs[i]);
  return s;
}

extern "C" uint64_t sdx_exchange_send_bytes(const sdx_xchg_part* parts, int k) {
  uint64_t s = 0;
  for (int i = 0; i < k; ++i)
    if (!parts[i].aux) s += r16(4ull * parts[i].n_msgs) + r16(8ull * parts[i].rec_cap) + r16(parts[i].heap_cap);
  // an overlaid launch may take its records from its overlays: their capacities bound its sections too
  for (int i = 0; i < k; ++i)
    if (parts[i].aux) s += r16(8ull * parts[i].rec_cap) + r16(parts[i].heap_cap);
  return s;
}

static int check_parts(const sdx_xchg_part* parts, int k, const char* who) {
  if (!parts || k < 1 || k > XMAX) return sdx::set_error(SDX_EINVAL, std::string(who) + ": 1..SDX_XCHG_MAX_PARTS launches");
  for (int i = 0; i < k; ++i) {
    const sdx_xchg_part& x = parts[i];
    if (!x.cursor_dev || (x.n_msgs && !x.desc_dev) || (x.rec_cap && !x.rec_dev) || (x.rec_cap && !x.heap_dev))
      return sdx::set_error(SDX_EINVAL, std::string(who) + ": missing buffer (records need a heap)");
    if (x.alt > k || x.alt == i + 1)
      return sdx::set_error(SDX_EINVAL, std::string(who) + ": overlay index out of range");
    if (x.alt && (!parts[x.alt - 1].aux || parts[x.alt - 1].n_msgs != x.n_msgs))
      return sdx::set_error(SDX_EINVAL, std::string(who) + ": an overlay must be aux and cover the same messages");
  }
  return SDX_OK;
}

static Parts make_parts(const sdx_bank* bank, const sdx_xchg_part* parts, int k) {
  Parts P;
  uint64_t off = 0;
  P.k = k;
  P.shared = 0;
  P.bank = bank ? reinterpret_cast<const uint8_t*>(sdx::bank_dev_ptr(bank)) : nullptr;
  for (int i = 0; i < XMAX; ++i) {
    P.p[i] = i < k ? parts[i] : sdx_xchg_part{};
    P.work_off[i] = off;
    P.owner[i] = -1;
    if (i < k) off += part_work_bytes(parts[i].n_msgs);
  }
  for (int i = 0; i < k; ++i) {  // each launch and the overlays along its chain (resolve's walk)
    if (parts[i].aux) continue;
    P.owner[i] = i;
    for (int c = i, hop = 0; hop < CHAIN; ++hop) {
      const int a = (int)parts[c].alt - 1;
      if (a < 0 || a >= k) break;
      if (P.owner[a] < 0) P.owner[a] = i;
      else if (P.owner[a] != i) P.shared = 1;
      c = a;
    }
  }
  return P;
}

static int launched(const char* name) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string(name) + ": " + hipGetErrorString(e));
  return SDX_OK;
}

static bool work_ok(const sdx_xchg_part* parts, int k, const void* work_dev, uint64_t work_cap) {
  uint32_t ns[XMAX];
  for (int i = 0; i < k; ++i) ns[i] = parts[i].n_msgs;
  return work_dev && ((uintptr_t)work_dev & 255u) == 0 && work_cap >= sdx_exchange_work_bytes(ns, k);
}

static uint32_t max_blocks(const sdx_xchg_part* parts, int k) {
  uint32_t nb = 1;
  for (int i = 0; i < k; ++i) nb = nblk_of(parts[i].n_msgs) > nb ? nblk_of(parts[i].n_msgs) : nb;
  return nb;
}

// the pack: SDX_XCHG_PACK_MSG=1 in the environment selects the message-order k_xw_pack (A/B);
// otherwise k_xw_words + k_xw_recs (the same bytes, source-record order)
static int launch_pack(const sdx_bank* bank, const sdx_xchg_part* parts, int k, const uint32_t* counts_dev,
                       const uint32_t* counts_host, uint8_t* work, uint8_t* dst, hipStream_t st) {
  const char* e = getenv("SDX_XCHG_PACK_MSG");  // read per call: a test compares both forms in one process
  const bool msg_order = e && e[0] == '1';
  const Parts P = make_parts(bank, parts, k);
  if (msg_order || P.shared) {  // (an overlay shared by two launches: the message-order pack resolves it)
    hipLaunchKernelGGL(k_xw_pack, dim3(max_blocks(parts, k), k), dim3(XT), 0, st, P, counts_dev, work, dst);
    return launched("k_xw_pack");
  }
  hipLaunchKernelGGL(k_xw_words, dim3(max_blocks(parts, k), k), dim3(XT), 0, st, P, counts_dev, work, dst);
  if (int rc = launched("k_xw_words")) return rc;
  // record blocks: one per 256 records of the largest part's capacity, or, with the host's copy of the
  // counts, of the largest launch's shipped records (plus one block): the blocks past a part's cursor
  // return at once but still cost their dispatch (47k of them for the bench step's capacities), and
  // records past the grid (overlays, records not shipped) are taken by the grid-stride loop.  (A
  // grid of 1024 blocks per part measured slower: 87.7 vs 70.3 us for the bench step.)
  uint32_t nbr = 1;
  for (int i = 0; i < k; ++i) {
    const uint32_t nb = counts_host ? nblk_of(counts_host[SDX_XCHG_COUNTS * i + 1]) + 1 : nblk_of(parts[i].rec_cap);
    nbr = nb > nbr ? nb : nbr;
  }
  nbr = nbr < XREC_GRID ? nbr : XREC_GRID;
  hipLaunchKernelGGL(k_xw_recs, dim3(nbr, k), dim3(XT), 0, st, P, counts_dev, work, dst);
  return launched("k_xw_recs");
}

extern "C" int sdx_exchange_count(const sdx_bank* bank, const sdx_xchg_part* parts, int k, void* work_dev,
                                  uint64_t work_cap, uint32_t* counts_dev, void* hip_stream) {
  if (int rc = check_parts(parts, k, "sdx_exchange_count")) return rc;
  if (!counts_dev || !work_ok(parts, k, work_dev, work_cap))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_count: workspace too small / unaligned, or no counts buffer");
  const Parts P = make_parts(bank, parts, k);
  hipLaunchKernelGGL(k_xw_count, dim3(max_blocks(parts, k), k), dim3(XT), 0, (hipStream_t)hip_stream, P,
                     (uint8_t*)work_dev);
  if (int rc = launched("k_xw_count")) return rc;
  hipLaunchKernelGGL(k_xw_scan, dim3(k), dim3(XT), 0, (hipStream_t)hip_stream, P, (uint8_t*)work_dev, counts_dev);
  return launched("k_xw_scan");
}

extern "C" int sdx_exchange_pack(const sdx_bank* bank, const sdx_xchg_part* parts, int k, void* work_dev,
                                 uint64_t work_cap, const uint32_t* counts_dev, uint8_t* send_dev, uint64_t send_cap,
                                 void* hip_stream) {
  if (int rc = check_parts(parts, k, "sdx_exchange_pack")) return rc;
  if (!counts_dev || !send_dev || ((uintptr_t)send_dev & 15u) || send_cap < sdx_exchange_send_bytes(parts, k) ||
      !work_ok(parts, k, work_dev, work_cap))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack: workspace or send buffer too small / unaligned");
  return launch_pack(bank, parts, k, counts_dev, nullptr, (uint8_t*)work_dev, send_dev, (hipStream_t)hip_stream);
}

// the pack into a buffer sized from the host's copy of the counts (the exact layout), e.g. the rank's
// own chunk of an in-place all-gather's receive buffer
extern "C" int sdx_exchange_pack_into(const sdx_bank* bank, const sdx_xchg_part* parts, int k, void* work_dev,
                                      uint64_t work_cap, const uint32_t* counts_dev, const uint32_t* counts_host,
                                      uint8_t* dst_dev, uint64_t dst_cap, void* hip_stream) {
  if (int rc = check_parts(parts, k, "sdx_exchange_pack_into")) return rc;
  if (!counts_dev || !counts_host || !dst_dev || ((uintptr_t)dst_dev & 15u) || !work_ok(parts, k, work_dev, work_cap))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack_into: missing / unaligned buffer or workspace too small");
  uint64_t need = 0;
  for (int i = 0; i < k; ++i) {
    const uint32_t* c = counts_host + SDX_XCHG_COUNTS * i;
    if (c[0] != (parts[i].aux ? 0u : parts[i].n_msgs))
      return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack_into: counts_host are not this exchange's counts");
    need += r16(4ull * c[0]) + r16(8ull * c[1]) + r16(c[2]);
  }
  if (dst_cap < need) return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack_into: destination smaller than the wire");
  return launch_pack(bank, parts, k, counts_dev, counts_host, (uint8_t*)work_dev, dst_dev, (hipStream_t)hip_stream);
}

extern "C" uint64_t sdx_exchange_unpack_work_bytes(uint32_t n_msgs, uint32_t n_rec) {
  return 64 + 8ull * (nblk_of(n_msgs) + nblk_of(n_rec)) + 4ull * n_rec;
}

extern "C" int sdx_exchange_unpack(const sdx_bank* bank, int kind, const sdx_xchg_wire* ranks, int nranks,
                                   void* work_dev, uint64_t work_cap, sdx_desc* desc_dev, sdx_result* rec_dev,
                                   uint8_t* heap_dev, uint64_t heap_cap, void* hip_stream) {
  if (!ranks || nranks < 1 || nranks > XRANKS)
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: 1..SDX_XCHG_MAX_RANKS ranks");
  Wire W;
  W.nranks = nranks;
  W.kind = kind;
  W.bank = bank ? reinterpret_cast<const uint8_t*>(sdx::bank_dev_ptr(bank)) : nullptr;
  uint64_t m = 0, r = 0, h = 0, pay = 0;
  // every prefix entry [0, XRANKS] is written: the ranks' starts, then the end sentinel at [nranks]
  // and beyond (the kernels read [nranks] as the job's totals, also when nranks == XRANKS)
  for (int i = 0; i <= XRANKS; ++i) {
    if (i < XRANKS) W.r[i] = i < nranks ? ranks[i] : sdx_xchg_wire{};
    W.msg0[i] = (uint32_t)m;
    W.rec0[i] = (uint32_t)r;
    W.wire0[i] = (uint32_t)h;
    if (i < nranks) {
      m += ranks[i].n_msgs;
      r += ranks[i].n_rec;
      h += ranks[i].n_heap;
      pay += ranks[i].n_payload;
      if ((ranks[i].n_msgs && !ranks[i].msg_dev) || (ranks[i].n_rec && !ranks[i].rec_dev) ||
          (ranks[i].n_heap && !ranks[i].heap_dev))
        return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: missing section");
    }
  }
  if (m >= (1ull << 32) || r >= (1ull << 31) || h >= (1ull << 31) || pay >= (1ull << 32))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: the job exceeds 32-bit message / record / heap indices");
  if (!work_dev || work_cap < sdx_exchange_unpack_work_bytes((uint32_t)m, (uint32_t)r) || ((uintptr_t)work_dev & 63u) ||
      (m && !desc_dev) || (r && !rec_dev) || (pay && !heap_dev) || heap_cap < pay)
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: bad workspace or output buffers (heap_cap < payload bytes)");
  const uint32_t nb = nblk_of(m) + nblk_of(r);
  hipStream_t st = (hipStream_t)hip_stream;
  hipLaunchKernelGGL(k_xu_sum, dim3(nb), dim3(XT), 0, st, W, (uint8_t*)work_dev);
  if (int rc = launched("k_xu_sum")) return rc;
  hipLaunchKernelGGL(k_xu_scan, dim3(1), dim3(XT), 0, st, W, (uint8_t*)work_dev);
  if (int rc = launched("k_xu_scan")) return rc;
  hipLaunchKernelGGL(k_xu_write, dim3(nb), dim3(XT), 0, st, W, (uint8_t*)work_dev, desc_dev, rec_dev);
  if (int rc = launched("k_xu_write")) return rc;
  if (r) {
    hipLaunchKernelGGL(k_xu_heap, dim3((uint32_t)((r + XT - 1) / XT)), dim3(XT), 0, st, W, (const uint8_t*)work_dev,
                       rec_dev, heap_dev);
    if (int rc = launched("k_xu_heap")) return rc;
  }
  return SDX_OK;
}
