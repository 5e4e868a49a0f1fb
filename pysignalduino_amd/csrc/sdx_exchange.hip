// sdx_exchange.hip -- the device side of the multi-GPU exchange (BASELINE config 5).
//
// Every rank demodulates its contiguous shard of the stream; the one exchange step all-gathers the
// decoded dmsg buffers of all ranks over RCCL.  What travels is the wire form of include/sdx.h:
// per launch and rank, in message order, a 4-byte word per message (n_rec, status, raise_kind), an
// 8-byte sdx_wire_rec per record (proto, payload_len, bit_length) and the payloads concatenated.
// rec_begin, payload_off and msg are prefix sums and are not sent: 4 + 8 * records + payload bytes
// per message instead of 8 + 16 * records + the (padded) heap.
//
// Sender, two launches around the host's count exchange:
//   k_xw_count  lane = 4 consecutive messages: validate each descriptor and its records against the
//               launch's cursor / capacities, count records and payload bytes, block-scan them
//               (per-message local prefixes into the workspace); the last block of a launch to
//               finish scans the block totals and publishes the launch's counts (no inter-block
//               waiting: a block that is not last just leaves).
//   k_xw_pack   lane = message (its wire word) and lane = source record (its wire record at the
//               message's prefix + its rank in the message, and its payload bytes).  The source
//               records are in tile order (k_pulses places them per tile); the wire is in message
//               order, so the pack is also the canonicalisation that makes sharded and un-sharded
//               runs compare byte for byte.
// Receiver:
//   k_xu_scan / k_xu_write  rebuild sdx_desc / sdx_result / one contiguous heap of the whole job from
//               the gathered wire sections of every rank (the same last-block scan, over the
//               rank-concatenated messages and records).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/sdx.h"

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
}

namespace sdxx {

constexpr int XT = 256;       // threads per block
constexpr int IPT = 1;        // items per thread in the scans (one message: its loads all in flight)
constexpr int XB = XT * IPT;  // items per block
constexpr int XMAX = 8;       // launches per exchange
constexpr int XRANKS = SDX_XCHG_MAX_RANKS;
constexpr uint64_t BADBIT = 1ull << 63;

__host__ __device__ inline uint32_t nblk_of(uint64_t n) { return n ? (uint32_t)((n + XB - 1) / XB) : 1u; }
__host__ __device__ inline uint64_t r16(uint64_t x) { return (x + 15) & ~15ull; }
// workspace: header (256 B: launches done, the send layout) | per launch: [ctr, bad, tot[2]] (64 B),
// loc u64[n], blk u64[nblk]
constexpr uint64_t HDR = 256;
__host__ __device__ inline uint64_t part_work_bytes(uint32_t n) {
  return (64 + 8ull * n + 8ull * nblk_of(n) + 255) / 256 * 256;
}

struct Parts {
  sdx_xchg_part p[XMAX];
  uint64_t work_off[XMAX];
  int k;
};

struct Hdr {
  uint32_t done;             // launches whose count finished (reset by the last)
  uint32_t res;
  uint64_t off[XMAX][3];     // the send layout: msg / rec / heap section offsets per launch
  uint64_t total;
};

struct PartWork {
  uint32_t* ctr;   // blocks done (reset by the last block)
  uint32_t* bad;   // bad messages (reset by the last block)
  uint32_t* tot;   // [2]: records, payload bytes of the launch (read by k_xw_pack)
  uint64_t* loc;   // per message: BADBIT | local record prefix << 32 | local byte prefix
  uint64_t* blk;   // block totals -> exclusive block offsets (records << 32 | bytes)
};

__device__ inline PartWork part_work(uint8_t* work, uint64_t off, uint32_t n) {
  PartWork w;
  uint8_t* b = work + HDR + off;
  w.ctr = reinterpret_cast<uint32_t*>(b);
  w.bad = w.ctr + 1;
  w.tot = w.ctr + 2;
  w.loc = reinterpret_cast<uint64_t*>(b + 64);
  w.blk = w.loc + n;
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

// in-place exclusive scan of blk[0, nb) by one block (after an acquire fence); returns the sum
__device__ inline uint64_t block_scan_array(uint64_t* blk, uint32_t nb) {
  uint64_t carry = 0;
  for (uint32_t c = 0; c < nb; c += XT) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < nb ? __hip_atomic_load(&blk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    uint64_t tot;
    const uint64_t ex = block_excl(v, &tot);
    if (i < nb) blk[i] = carry + ex;
    carry += tot;
  }
  return carry;
}

// last-block protocol: publish this block's total, count the block in; true in every thread of the
// block that finished last (which then sees every block's total after its acquire fence)
__device__ inline bool arrive_last(uint64_t* blk_slot, uint64_t total, uint32_t* ctr, uint32_t nb) {
  __shared__ bool s_last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(blk_slot, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    s_last = atomicAdd(ctr, 1u) == nb - 1;
  }
  __syncthreads();
  if (s_last) __threadfence();
  return s_last;
}

__device__ inline void clamp_counts(const sdx_xchg_part& x, uint32_t* nrec_c, uint32_t* nheap_c) {
  const uint32_t c0 = x.cursor_dev[0], c1 = x.cursor_dev[1];
  *nrec_c = c0 < x.rec_cap ? c0 : x.rec_cap;
  *nheap_c = c1 < x.heap_cap ? c1 : x.heap_cap;
}

// the validated (records << 32 | payload bytes) of message m; *ok = false marks a message the
// exchange cannot ship (an overflow status, or a descriptor / record outside what the launch wrote)
__device__ inline uint64_t msg_counts(const sdx_xchg_part& x, uint32_t nrec_c, uint32_t nheap_c, uint32_t m,
                                      bool* ok) {
  const sdx_desc d = reinterpret_cast<const sdx_desc*>(x.desc_dev)[m];
  *ok = true;
  if (d.status == SDX_ST_RAISED) return 0;
  if (d.status != SDX_ST_OK || (d.n_rec && (uint64_t)d.rec_begin + d.n_rec > nrec_c)) {
    *ok = false;
    return 0;
  }
  const sdx_result* r = reinterpret_cast<const sdx_result*>(x.rec_dev) + d.rec_begin;
  uint64_t bytes = 0;
  bool good = true;
#pragma unroll 4
  for (uint32_t j = 0; j < d.n_rec; ++j) {
    const sdx_result v = r[j];
    good &= v.msg == m && (uint64_t)v.payload_off + v.payload_len <= nheap_c;
    bytes += v.payload_len;
  }
  *ok = good;
  return good ? (((uint64_t)d.n_rec << 32) | bytes) : 0;
}

// the send layout, in launch order: [msg | rec | heap] sections of each launch, 16-byte aligned
__device__ inline void make_layout(Hdr* h, const uint32_t* counts, int K) {
  uint64_t off = 0;
  for (int k = 0; k < K; ++k) {
    h->off[k][0] = off;
    off += r16(4ull * counts[4 * k]);
    h->off[k][1] = off;
    off += r16(8ull * counts[4 * k + 1]);
    h->off[k][2] = off;
    off += r16(counts[4 * k + 2]);
  }
  h->total = off;
}

__global__ __launch_bounds__(XT) void k_xw_count(Parts P, uint8_t* __restrict__ work, uint32_t* __restrict__ counts) {
  const int k = blockIdx.y;
  const sdx_xchg_part& x = P.p[k];
  const uint32_t nb = nblk_of(x.n_msgs);
  if (blockIdx.x >= nb) return;
  PartWork w = part_work(work, P.work_off[k], x.n_msgs);
  uint32_t nrec_c, nheap_c;
  clamp_counts(x, &nrec_c, &nheap_c);
  const uint32_t m = blockIdx.x * XB + threadIdx.x;
  bool ok = true;
  uint64_t v = m < x.n_msgs ? msg_counts(x, nrec_c, nheap_c, m, &ok) : 0;
  uint64_t tot;
  const uint64_t pre = block_excl(v, &tot);
  if (m < x.n_msgs) w.loc[m] = pre | (ok ? 0 : BADBIT);
  const uint64_t bad_wave = __ballot(!ok);
  if (lane_id() == 0 && bad_wave) atomicAdd(w.bad, (uint32_t)__popcll(bad_wave));
  if (!arrive_last(&w.blk[blockIdx.x], tot, w.ctr, nb)) return;
  const uint64_t all = block_scan_array(w.blk, nb);
  __shared__ bool s_lastk;
  if (threadIdx.x == 0) {
    const uint32_t bd = __hip_atomic_load(w.bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w.tot[0] = (uint32_t)(all >> 32);
    w.tot[1] = (uint32_t)all;
    counts[4 * k + 0] = x.n_msgs;
    counts[4 * k + 1] = (uint32_t)(all >> 32);
    counts[4 * k + 2] = (uint32_t)all;
    counts[4 * k + 3] = bd;
    *w.bad = 0;
    *w.ctr = 0;
    // the launch that finishes last lays out the send buffer from every launch's counts
    Hdr* h = reinterpret_cast<Hdr*>(work);
    __threadfence();
    s_lastk = atomicAdd(&h->done, 1u) == (uint32_t)P.k - 1;
    if (s_lastk) {
      __threadfence();
      uint32_t c[4 * XMAX];
      for (int i = 0; i < 4 * P.k; ++i) c[i] = __hip_atomic_load(&counts[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      make_layout(h, c, P.k);
      h->done = 0;
    }
  }
}

// copy n payload bytes (arbitrary alignment on both sides): 16 independent byte loads in flight per
// step, then their stores
__device__ inline void copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t n) {
  for (uint32_t c = 0; c < n; c += 16) {
    uint8_t b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = c + i < n ? src[c + i] : 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (c + i < n) dst[c + i] = b[i];
  }
}

__device__ inline void zero_tail(uint8_t* sec, uint64_t used, uint32_t lane) {
  if (lane < 16 && used + lane < r16(used)) sec[used + lane] = 0;
}

// lane = message (grid-stride), grid.y = launch: the message's wire word, its records (contiguous in
// the source, from rec_begin) as wire records at its record prefix, its payloads at its byte prefix
__global__ __launch_bounds__(XT) void k_xw_pack(Parts P, const uint8_t* __restrict__ work, uint8_t* __restrict__ send) {
  const int k = blockIdx.y;
  const sdx_xchg_part& x = P.p[k];
  const Hdr* h = reinterpret_cast<const Hdr*>(work);
  PartWork w = part_work(const_cast<uint8_t*>(work), P.work_off[k], x.n_msgs);
  uint8_t* s_msg = send + h->off[k][0];
  sdx_wire_rec* s_rec = reinterpret_cast<sdx_wire_rec*>(send + h->off[k][1]);
  uint8_t* s_heap = send + h->off[k][2];
  const uint32_t g0 = blockIdx.x * XT + threadIdx.x;
  if (blockIdx.x == 0) {  // deterministic section padding
    zero_tail(s_msg, 4ull * x.n_msgs, threadIdx.x);
    zero_tail(reinterpret_cast<uint8_t*>(s_rec), 8ull * w.tot[0], threadIdx.x);
    zero_tail(s_heap, w.tot[1], threadIdx.x);
  }
  const sdx_desc* desc = reinterpret_cast<const sdx_desc*>(x.desc_dev);
  const sdx_result* rec = reinterpret_cast<const sdx_result*>(x.rec_dev);
  for (uint32_t m = g0; m < x.n_msgs; m += gridDim.x * XT) {
    const sdx_desc d = desc[m];
    const uint64_t loc = w.loc[m];
    const uint64_t base = w.blk[m / XB] + (loc & ~BADBIT);
    const bool bad = (loc & BADBIT) != 0;
    const uint32_t nr = (bad || d.status != SDX_ST_OK) ? 0u : d.n_rec;
    reinterpret_cast<uint32_t*>(s_msg)[m] =
        nr | ((uint32_t)(bad ? SDX_ST_OVF_OUT : d.status) << 16) | ((uint32_t)d.raise_kind << 24);
    uint32_t ri = (uint32_t)(base >> 32), byte = (uint32_t)base;
    for (uint32_t j = 0; j < nr; j += 4) {
      sdx_result r4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (j + i < nr) r4[i] = rec[d.rec_begin + j + i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (j + i >= nr) break;
        sdx_wire_rec o;
        o.proto = r4[i].proto;
        o.payload_len = r4[i].payload_len;
        o.bit_length = r4[i].bit_length;
        s_rec[ri++] = o;
        copy_bytes(s_heap + byte, x.heap_dev + r4[i].payload_off, r4[i].payload_len);
        byte += r4[i].payload_len;
      }
    }
  }
}

// ---- receiver ------------------------------------------------------------------------------------
struct Wire {
  sdx_xchg_wire r[XRANKS];
  uint32_t msg0[XRANKS + 1];   // first global message of rank r
  uint32_t rec0[XRANKS + 1];   // first global record
  uint32_t heap0[XRANKS + 1];  // first global payload byte
  int nranks;
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

// items: global messages [0, M) (value: records << 32) in blocks [0, nbm), global records [0, R)
// (value: payload bytes) in blocks [nbm, nbm + nbr)
__device__ inline uint64_t xu_item(const Wire& W, bool is_msg, uint32_t g, uint32_t M, uint32_t R) {
  if (is_msg) {
    if (g >= M) return 0;
    const int r = rank_of(W.msg0, W.nranks, g);
    const uint32_t word = reinterpret_cast<const uint32_t*>(W.r[r].msg_dev)[g - W.msg0[r]];
    return (uint64_t)(word & 0xffffu) << 32;
  }
  if (g >= R) return 0;
  const int r = rank_of(W.rec0, W.nranks, g);
  return reinterpret_cast<const sdx_wire_rec*>(W.r[r].rec_dev)[g - W.rec0[r]].payload_len;
}

__global__ __launch_bounds__(XT) void k_xu_scan(Wire W, uint8_t* __restrict__ work) {
  const uint32_t M = W.msg0[W.nranks], R = W.rec0[W.nranks];
  const uint32_t nbm = nblk_of(M), nbr = nblk_of(R);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(work);
  uint64_t* blk = reinterpret_cast<uint64_t*>(work + 64);
  const bool is_msg = blockIdx.x < nbm;
  const uint32_t b = is_msg ? blockIdx.x : blockIdx.x - nbm;
  const uint32_t g0 = b * XB + threadIdx.x * IPT;
  uint64_t sum = 0;
#pragma unroll
  for (int j = 0; j < IPT; ++j) sum += xu_item(W, is_msg, g0 + j, M, R);
  uint64_t tot;
  (void)block_excl(sum, &tot);
  if (!arrive_last(&blk[blockIdx.x], tot, ctr, nbm + nbr)) return;
  block_scan_array(blk, nbm);
  block_scan_array(blk + nbm, nbr);
  if (threadIdx.x == 0) *ctr = 0;
}

// blocks [0, nbm): descriptors (and each record's msg field); [nbm, nbm + nbr): records;
// then heap blocks: one output dword per thread
__global__ __launch_bounds__(XT) void k_xu_write(Wire W, const uint8_t* __restrict__ work, sdx_desc* __restrict__ desc,
                                                 sdx_result* __restrict__ rec, uint8_t* __restrict__ heap) {
  const uint32_t M = W.msg0[W.nranks], R = W.rec0[W.nranks], H = W.heap0[W.nranks];
  const uint32_t nbm = nblk_of(M), nbr = nblk_of(R);
  const uint64_t* blk = reinterpret_cast<const uint64_t*>(work + 64);
  if (blockIdx.x >= nbm + nbr) {  // heap: output dword d = bytes [4d, 4d + 4)
    const uint32_t d = (blockIdx.x - nbm - nbr) * XT + threadIdx.x;
    if (4ull * d >= H) return;
    uint32_t word = 0;
    int r = rank_of(W.heap0, W.nranks, 4 * d);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t p = 4 * d + i;
      if (p >= H) break;
      while (p >= W.heap0[r + 1]) ++r;
      word |= (uint32_t)W.r[r].heap_dev[p - W.heap0[r]] << (8 * i);
    }
    if (4ull * d + 4 <= H) {
      reinterpret_cast<uint32_t*>(heap)[d] = word;
    } else {
      for (uint32_t i = 0; 4 * d + i < H; ++i) heap[4 * d + i] = (uint8_t)(word >> (8 * i));
    }
    return;
  }
  const bool is_msg = blockIdx.x < nbm;
  const uint32_t b = is_msg ? blockIdx.x : blockIdx.x - nbm;
  const uint32_t g0 = b * XB + threadIdx.x * IPT;
  uint64_t v[IPT], sum = 0;
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    v[j] = xu_item(W, is_msg, g0 + j, M, R);
    sum += v[j];
  }
  uint64_t tot;
  uint64_t pre = block_excl(sum, &tot) + blk[blockIdx.x];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const uint32_t g = g0 + j;
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
      const int r = rank_of(W.rec0, W.nranks, g);
      const sdx_wire_rec wr = reinterpret_cast<const sdx_wire_rec*>(W.r[r].rec_dev)[g - W.rec0[r]];
      sdx_result* o = rec + g;
      o->payload_off = (uint32_t)pre;
      o->payload_len = wr.payload_len;
      o->proto = wr.proto;
      o->bit_length = wr.bit_length;
    }
    pre += v[j];
  }
}

}  // namespace sdxx

using namespace sdxx;

extern "C" uint64_t sdx_exchange_work_bytes(const uint32_t* n_msgs, int k) {
  uint64_t s = HDR;
  for (int i = 0; i < k; ++i) s += part_work_bytes(n_msgs[i]);
  return s;
}

extern "C" uint64_t sdx_exchange_send_bytes(const sdx_xchg_part* parts, int k) {
  uint64_t s = 0;
  for (int i = 0; i < k; ++i) s += r16(4ull * parts[i].n_msgs) + r16(8ull * parts[i].rec_cap) + r16(parts[i].heap_cap);
  return s;
}

static int check_parts(const sdx_xchg_part* parts, int k, const char* who) {
  if (!parts || k < 1 || k > XMAX) return sdx::set_error(SDX_EINVAL, std::string(who) + ": 1..8 launches");
  for (int i = 0; i < k; ++i) {
    const sdx_xchg_part& x = parts[i];
    if (!x.cursor_dev || (x.n_msgs && !x.desc_dev) || (x.rec_cap && !x.rec_dev) || (x.heap_cap && !x.heap_dev))
      return sdx::set_error(SDX_EINVAL, std::string(who) + ": missing buffer");
  }
  return SDX_OK;
}

static Parts make_parts(const sdx_xchg_part* parts, int k) {
  Parts P;
  uint64_t off = 0;
  P.k = k;
  for (int i = 0; i < XMAX; ++i) {
    P.p[i] = i < k ? parts[i] : sdx_xchg_part{};
    P.work_off[i] = off;
    if (i < k) off += part_work_bytes(parts[i].n_msgs);
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

extern "C" int sdx_exchange_count(const sdx_xchg_part* parts, int k, void* work_dev, uint64_t work_cap,
                                  uint32_t* counts_dev, void* hip_stream) {
  if (int rc = check_parts(parts, k, "sdx_exchange_count")) return rc;
  if (!counts_dev || !work_ok(parts, k, work_dev, work_cap))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_count: workspace too small / unaligned, or no counts buffer");
  uint32_t nbmax = 1;
  for (int i = 0; i < k; ++i) nbmax = nblk_of(parts[i].n_msgs) > nbmax ? nblk_of(parts[i].n_msgs) : nbmax;
  hipLaunchKernelGGL(k_xw_count, dim3(nbmax, k), dim3(XT), 0, (hipStream_t)hip_stream, make_parts(parts, k),
                     (uint8_t*)work_dev, counts_dev);
  return launched("k_xw_count");
}

extern "C" int sdx_exchange_pack(const sdx_xchg_part* parts, int k, void* work_dev, uint64_t work_cap,
                                 uint8_t* send_dev, uint64_t send_cap, void* hip_stream) {
  if (int rc = check_parts(parts, k, "sdx_exchange_pack")) return rc;
  if (!send_dev || ((uintptr_t)send_dev & 15u) || send_cap < sdx_exchange_send_bytes(parts, k) ||
      !work_ok(parts, k, work_dev, work_cap))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack: workspace or send buffer too small / unaligned");
  uint64_t most = 1;
  for (int i = 0; i < k; ++i) most = parts[i].n_msgs > most ? parts[i].n_msgs : most;
  uint64_t blocks = (most + XT - 1) / XT;
  blocks = blocks > 8192 ? 8192 : blocks;
  hipLaunchKernelGGL(k_xw_pack, dim3((unsigned)blocks, k), dim3(XT), 0, (hipStream_t)hip_stream,
                     make_parts(parts, k), (const uint8_t*)work_dev, send_dev);
  return launched("k_xw_pack");
}

extern "C" uint64_t sdx_exchange_unpack_work_bytes(uint32_t n_msgs, uint32_t n_rec) {
  return 64 + 8ull * (nblk_of(n_msgs) + nblk_of(n_rec));
}

extern "C" int sdx_exchange_unpack(const sdx_xchg_wire* ranks, int nranks, void* work_dev, uint64_t work_cap,
                                   sdx_desc* desc_dev, sdx_result* rec_dev, uint8_t* heap_dev, void* hip_stream) {
  if (!ranks || nranks < 1 || nranks > XRANKS)
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: 1..SDX_XCHG_MAX_RANKS ranks");
  Wire W;
  W.nranks = nranks;
  uint64_t m = 0, r = 0, h = 0;
  for (int i = 0; i < XRANKS; ++i) {
    W.r[i] = i < nranks ? ranks[i] : sdx_xchg_wire{};
    if (i <= nranks) {
      W.msg0[i] = (uint32_t)m;
      W.rec0[i] = (uint32_t)r;
      W.heap0[i] = (uint32_t)h;
    }
    if (i < nranks) {
      m += ranks[i].n_msgs;
      r += ranks[i].n_rec;
      h += ranks[i].n_heap;
      if ((ranks[i].n_msgs && !ranks[i].msg_dev) || (ranks[i].n_rec && !ranks[i].rec_dev) ||
          (ranks[i].n_heap && !ranks[i].heap_dev))
        return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: missing section");
    }
  }
  if (nranks < XRANKS) {
    W.msg0[nranks] = (uint32_t)m;
    W.rec0[nranks] = (uint32_t)r;
    W.heap0[nranks] = (uint32_t)h;
  }
  if (m >= (1ull << 32) || r >= (1ull << 32) || h >= (1ull << 32))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: the job exceeds 32-bit message / record / heap indices");
  if (!work_dev || work_cap < sdx_exchange_unpack_work_bytes((uint32_t)m, (uint32_t)r) || ((uintptr_t)work_dev & 63u) ||
      (m && !desc_dev) || (r && !rec_dev) || (h && !heap_dev) || ((uintptr_t)heap_dev & 3u))
    return sdx::set_error(SDX_EINVAL, "sdx_exchange_unpack: bad workspace or output buffers");
  const uint32_t nb = nblk_of(m) + nblk_of(r);
  const uint32_t nh = (uint32_t)((h + 4ull * XT - 1) / (4ull * XT));
  hipLaunchKernelGGL(k_xu_scan, dim3(nb), dim3(XT), 0, (hipStream_t)hip_stream, W, (uint8_t*)work_dev);
  if (int rc = launched("k_xu_scan")) return rc;
  hipLaunchKernelGGL(k_xu_write, dim3(nb + nh), dim3(XT), 0, (hipStream_t)hip_stream, W, (const uint8_t*)work_dev,
                     desc_dev, rec_dev, heap_dev);
  return launched("k_xu_write");
}
