// sdx_group.hip -- message grouping for k_pulses (MU / MS): a per-message key and a device radix
// sort that orders the batch by it.
//
// k_pulses runs its filter with lane = message and one protocol per wave (scalar bank records).
// The expensive part of pattern_exists (pattern_utils.py:86-136: combinations, substring searches)
// runs for a wave when ANY of its 64 messages has candidates for every value of the protocol's
// keys (the cheap first step, :53-80); on a random message order about a third of the lanes of
// such a wave do.  Sorting the messages by WHICH protocols they pass that cheap step puts messages
// with the same candidate protocols into one tile (the bench corpus runs 2.3x fewer
// wave-iterations of the expensive part, at 2.3x the lane occupancy).  The key only orders the
// work: every message still runs against the whole bank and results are placed by message index,
// so the output is identical (tests/test_gpu_parity.py runs both orders).  GPU tiles finish in any
// order anyway: consumers read results through the descriptors (sdx_desc.rec_begin / n_rec).
#include "sdx_device.h"
#include "sdx_lane.h"

namespace sdx {

// lanes below this one in `mask`
SDX_DEV int lanes_below_mask(uint64_t mask) {
  const int l = lane_id();
  return popc64(l ? (mask & ((1ull << l) - 1)) : 0ull);
}
// the lanes of the wave (among `active`) whose 8-bit value equals this lane's
SDX_DEV uint64_t peers8(uint32_t v, bool active) {
  uint64_t peers = ballot(active);
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) {
    const uint64_t bb = ballot(active && ((v >> bit) & 1u));
    peers &= ((v >> bit) & 1u) ? bb : ~bb;
  }
  return peers;
}

// ---------------------------------------------------------------------------------------------
// the key: bit 31 - r = the message passes the candidate-interval test of the first search list of
// protocol r (bank order, r < 32) -- start, else one, for MU after round(P / clockabs, 1)
// (message_unsynced.py:64); the clockabs gate and sync for MS (message_synced.py:64-88, 128).
// Lane = message; the protocol loop is uniform (scalar record loads).  (Measured on the bench
// corpus: the first list groups better than all of a protocol's lists, and bank order better than
// the clock-grouped processing order.)
// ---------------------------------------------------------------------------------------------
constexpr int SIG_PROTOS = 32;
#ifndef SDX_MS_LONG_FIRST
#define SDX_MS_LONG_FIRST 0  // 1: the MS length class of more than 128 pulses first (A/B)
#endif
#ifndef SDX_MS_KEY
#define SDX_MS_KEY 0  // MS key form (A/B experiments; 0 = ascending signature)
#endif
template <int KIND>
SDX_DEV void sig_block(const void* __restrict__ bank, const sdx_pulse_batch& b, uint32_t* __restrict__ key,
                       uint32_t* __restrict__ msg_out, sdx_msg_rec* __restrict__ mrec, const int blk) {
  const BankView bv = bank_view(bank);
  const int i = blk * 256 + threadIdx.x;
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const bool valid = i < ntot;
  const int msg = valid ? (b.sel_dev ? b.sel_dev[i] : i) : 0;
  int npat = valid ? b.npat_dev[msg] : 0;
  npat = npat > SDX_MAXPAT ? SDX_MAXPAT : npat;
  double val[SDX_MAXPAT];
#pragma unroll
  for (int k = 0; k < SDX_MAXPAT; ++k) val[k] = k < npat ? b.pat_val_dev[msg * SDX_MAXPAT + k] : 0.0;
  int kq[SDX_MAXPAT];
  uint32_t sig = 0;
  // the candidate test of one search list: every unique value has a slot in [klo, khi]
  auto keys_ok = [&](const SpecV& sv) -> bool {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < SDX_MAXUNIQ; ++u) {
      if (u < sv.nu) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < SDX_MAXPAT; ++j) any |= k_in(kq[j], sv.klo[u], sv.khi[u]);
        ok = ok && any;
      }
    }
    return ok;
  };
  if constexpr (KIND == SDX_KIND_MU) {
    // round(P / clockabs, 1) * 10 in fp32: the key only orders the work, so a value that lands on
    // the other side of an interval border than the exact fp64 test would costs nothing but grouping
    float x10[SDX_MAXPAT];
#pragma unroll
    for (int k = 0; k < SDX_MAXPAT; ++k) x10[k] = (float)(val[k] * 10.0);
    const int nr = (int)bv.hdr->n_mu < SIG_PROTOS ? (int)bv.hdr->n_mu : SIG_PROTOS;
    double last = __builtin_nan("");
    for (int r = 0; r < nr; ++r) {
      const sdx_mu_filt* fr = uniform_ptr(bv.mufilt + r);
      const sdx_mu_proto* rec = uniform_ptr(bv.mu + r);
      const uint32_t ff = cld(&fr->flags);
      bool ok = !(ff & 2u) && (ff & 4u);  // active, not never
      if (ok) {
        const double pclk = cld(&fr->clock);
        if (pclk != last) {
          last = pclk;
          const float inv = 1.0f / (float)pclk;
#pragma unroll
          for (int k = 0; k < SDX_MAXPAT; ++k) {
            const float q = x10[k] * inv;
            kq[k] = (k < npat && fabsf(q) < 1.0e8f) ? (int)rintf(q) : SDX_K_NONE;
          }
        }
        // the protocol's first search list: start if it has one, else one (the list whose test
        // decides most often whether k_pulses runs the expensive search for the pair)
        const bool full = (ff & 8u) != 0;
        const int k = (ff & 1u) ? 0 : 1;
        const SpecV sv = full ? spec_full(k == 0 ? &rec->start : &rec->one)
                              : spec_compact(&fr->spec[k], k == 0 ? cld(&fr->start_upk) : (uint64_t)cld(&fr->spec[k].upk));
        if (sv.slen) ok = ok && keys_ok(sv);
      }
      sig |= (uint32_t)ok << (31 - r);
    }
  } else {
    const int cp = valid ? b.cp_slot_dev[msg] : -1;
    double clock = 0.0;
#pragma unroll
    for (int k = 0; k < SDX_MAXPAT; ++k)
      if (k == cp) clock = fabs(val[k]);
    const bool gate = valid && b.ms_ok_dev[msg] && cp >= 0 && cp < npat && clock != 0.0;
    const float inv = clock != 0.0 ? (float)(10.0 / clock) : 0.0f;  // fp32 is enough for a grouping key
#pragma unroll
    for (int k = 0; k < SDX_MAXPAT; ++k) {
      const float q = (float)val[k] * inv;
      kq[k] = (gate && k < npat && fabsf(q) < 1.0e8f) ? (int)rintf(q) : SDX_K_NONE;
    }
    const int nr = (int)bv.hdr->n_ms < SIG_PROTOS ? (int)bv.hdr->n_ms : SIG_PROTOS;
    for (int r = 0; r < nr; ++r) {
      const sdx_ms_filt* fr = uniform_ptr(bv.msfilt + r);
      const sdx_ms_proto* rec = uniform_ptr(bv.ms + r);
      const uint32_t ff = cld(&fr->flags);
      bool ok = gate && !(ff & 2u);
      const double pclk = cld(&fr->pclock);
      if (ok && pclk > 0.0) ok = !(fabs(pclk - clock) > clock * 0.3);
      if (ok) {  // the sync list (searched first, message_synced.py:128-143)
        const bool full = (ff & 8u) != 0;
        const SpecV sv = full ? spec_full(&rec->key[0]) : spec_compact(&fr->spec[0], cld(&fr->sync_upk));
        if (sv.slen) ok = ok && keys_ok(sv);
      }
      sig |= (uint32_t)ok << (31 - r);
    }
  }
  if (valid && mrec) {  // the message's 128-byte record (sdx_msg_rec), eight 16-byte stores
    const int64_t off = b.offsets_dev[msg];
    const int32_t len = b.len_dev ? b.len_dev[msg] : (int32_t)(b.offsets_dev[msg + 1] - off);
    uint32_t id[4] = {0, 0, 0, 0};  // bytes 16..31: pat_id[10], then zeros
#pragma unroll
    for (int k = 0; k < SDX_MAXPAT; ++k) id[k >> 2] |= (uint32_t)b.pat_id_dev[msg * SDX_MAXPAT + k] << (8 * (k & 3));
    const uint32_t w3 = (uint32_t)(valid ? b.npat_dev[msg] : 0) |
                        ((uint32_t)(uint8_t)(KIND == SDX_KIND_MS ? b.cp_slot_dev[msg] : -1) << 8) |
                        ((uint32_t)(KIND == SDX_KIND_MS ? b.ms_ok_dev[msg] : 0) << 16);
    uint4* d = reinterpret_cast<uint4*>(mrec + msg);
    d[0] = make_uint4((uint32_t)off, (uint32_t)((uint64_t)off >> 32), (uint32_t)len, w3);
    d[1] = make_uint4(id[0], id[1], id[2], 0u);
#pragma unroll
    for (int h = 0; h < SDX_MAXPAT / 2; ++h) {
      const uint64_t a = (uint64_t)__double_as_longlong(val[2 * h]), c = (uint64_t)__double_as_longlong(val[2 * h + 1]);
      d[2 + h] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)c, (uint32_t)(c >> 32));
    }
    d[7] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (valid) {
    // MU: descending signature order -- messages that pass the leading protocols, the tiles that
    // run the expensive search most, start first and the cheap tiles fill the kernel's tail
    // (MU 1.29 -> 1.21 ms; popcount-first keys measured 1.24 ms); MS measured better ascending
#if SDX_MS_KEY == 1
    const uint32_t ms_key = ~sig;
#elif SDX_MS_KEY == 2  // survivor count descending, then signature
    const uint32_t ms_key = ((uint32_t)(32 - popc64(sig)) << 26) | (sig >> 6);
#elif SDX_MS_KEY == 3  // survivor count ascending, then signature
    const uint32_t ms_key = ((uint32_t)popc64(sig) << 26) | (sig >> 6);
#else
    // (SDX_MS_NARROW: the top bit = the length class of sdx_demod_pulses' MS launches, more than 128
    // pulses, so each class's tiles come together, the signature below it)
    uint32_t ms_key = sig;
    if (SDX_MS_NARROW) {
      const int64_t o = b.offsets_dev[msg];
      const int len = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - o);
      ms_key = (((len > 128) != (SDX_MS_LONG_FIRST != 0)) ? 0x80000000u : 0u) | (sig >> 1);
    }
#endif
    key[i] = KIND == SDX_KIND_MU ? ~sig : ms_key;
    msg_out[i] = (uint32_t)msg;
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void k_sig(const void* __restrict__ bank, sdx_pulse_batch b, uint32_t* __restrict__ key,
                                             uint32_t* __restrict__ msg_out, sdx_msg_rec* __restrict__ mrec) {
  sig_block<KIND>(bank, b, key, msg_out, mrec, (int)blockIdx.x);
}

// the step's two groupings in one launch (sdx_group_step): blocks [0, g_mu) key the MU batch, the rest
// the MS batch
struct SigSide {
  sdx_pulse_batch b;
  uint32_t* key;
  uint32_t* msg;
  sdx_msg_rec* mrec;
};
__global__ __launch_bounds__(256) void k_sig2(const void* __restrict__ bank, SigSide mu, SigSide ms, int g_mu) {
  if ((int)blockIdx.x < g_mu)
    sig_block<SDX_KIND_MU>(bank, mu.b, mu.key, mu.msg, mu.mrec, (int)blockIdx.x);
  else
    sig_block<SDX_KIND_MS>(bank, ms.b, ms.key, ms.msg, ms.mrec, (int)blockIdx.x - g_mu);
}

// ---------------------------------------------------------------------------------------------
// stable LSD radix sort of (key, message) pairs: 4 passes of 8 bits over partitions of RS_PART
// elements; per pass the partitions' digit counts (k_rs_hist), their prefix over the partitions (a
// wave per digit, k_rs_scan_rows) and the scatter (k_rs_scatter, which also scans the 256 digit
// totals).  No inter-workgroup waiting: a decoupled look-back sort is latency-bound at these sizes.
// ---------------------------------------------------------------------------------------------
constexpr int RS_T = 512, RS_ROUNDS = 4, RS_PART = RS_T * RS_ROUNDS;
#ifndef SDX_RS_PASSES
#define SDX_RS_PASSES 4
#endif
#ifndef SDX_RS_PASSES_MS
#define SDX_RS_PASSES_MS SDX_RS_PASSES
#endif
constexpr int RS_PASSES = SDX_RS_PASSES;  // bytes of the key sorted on, from the top
constexpr int RS_PASSES_MS = SDX_RS_PASSES_MS;  // (MS: A/B)
static_assert(RS_PASSES >= 1 && RS_PASSES <= 4 && RS_PASSES_MS >= 1 && RS_PASSES_MS <= 4, "1..4 radix passes");

// hist[digit * np + part] = elements of the partition with that digit in pass d
SDX_DEV void rs_hist(const uint32_t* __restrict__ key, int n, int np, int d, uint32_t* __restrict__ hist, const int p,
                     uint32_t* c) {
  const int tid = threadIdx.x;
  if (tid < 256) c[tid] = 0;
  __syncthreads();
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int e = p * RS_PART + r * RS_T + tid;
    const bool valid = e < n;
    const uint32_t dig = valid ? (key[e] >> (8 * d)) & 255u : 0u;
    const uint64_t peers = peers8(dig, valid);
    if (valid && lane_id() == ffs64(peers)) atomicAdd(&c[dig], (uint32_t)popc64(peers));
  }
  __syncthreads();
  if (tid < 256) hist[(size_t)tid * np + p] = c[tid];
}
__global__ __launch_bounds__(RS_T) void k_rs_hist(const uint32_t* __restrict__ key, int n, int np, int d,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t c[256];
  rs_hist(key, n, np, d, hist, (int)blockIdx.x, c);
}

// each digit's row: exclusive prefix over the partitions (one wave per row); tot[digit] = total
SDX_DEV void rs_scan_rows(uint32_t* __restrict__ hist, int np, uint32_t* __restrict__ tot, const int blk) {
  const int row = blk * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t* h = hist + (size_t)row * np;
  uint32_t run = 0;
  for (int b0 = 0; b0 < np; b0 += 64) {
    const int x = b0 + lane;
    const uint32_t v = x < np ? h[x] : 0u;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (x < np) h[x] = run + incl - v;
    run += __shfl(incl, 63);
  }
  if (lane == 0) tot[row] = run;
}
__global__ __launch_bounds__(256) void k_rs_scan_rows(uint32_t* __restrict__ hist, int np, uint32_t* __restrict__ tot) {
  rs_scan_rows(hist, np, tot, (int)blockIdx.x);
}

// pass d: every partition scatters its elements, in order (stable), to
// (digit base = prefix of the digit totals) + (row offset of the partition) + (rank inside it)
SDX_DEV void rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, int n, int np, int d,
                        const uint32_t* __restrict__ hist, const uint32_t* __restrict__ tot, uint32_t* __restrict__ kout,
                        uint32_t* __restrict__ vout, const int p, uint32_t* run, uint32_t (*wc)[256]) {
  const int tid = threadIdx.x, wave = tid >> 6;
  const uint32_t t = tid < 256 ? tot[tid] : 0u;
  if (tid < 256) run[tid] = t;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive scan of the digit totals
    const uint32_t y = (tid < 256 && tid >= o) ? run[tid - o] : 0u;
    __syncthreads();
    if (tid < 256) run[tid] += y;
    __syncthreads();
  }
  if (tid < 256) run[tid] = run[tid] - t + hist[(size_t)tid * np + p];
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int e = p * RS_PART + r * RS_T + tid;
    const bool valid = e < n;
    const uint32_t k = valid ? kin[e] : 0u;
    const uint32_t v = valid ? vin[e] : 0u;
    const uint32_t dig = (k >> (8 * d)) & 255u;
    for (int x = tid; x < RS_T / 64 * 256; x += RS_T) (&wc[0][0])[x] = 0;
    __syncthreads();
    const uint64_t peers = peers8(dig, valid);
    if (valid && lane_id() == ffs64(peers)) wc[wave][dig] = (uint32_t)popc64(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = run[dig] + (uint32_t)lanes_below_mask(peers);
      for (int w = 0; w < wave; ++w) pos += wc[w][dig];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    if (tid < 256) {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < RS_T / 64; ++w) add += wc[w][tid];
      run[tid] += add;
    }
    __syncthreads();
  }
}
__global__ __launch_bounds__(RS_T) void k_rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                     int n, int np, int d, const uint32_t* __restrict__ hist,
                                                     const uint32_t* __restrict__ tot, uint32_t* __restrict__ kout,
                                                     uint32_t* __restrict__ vout) {
  __shared__ uint32_t run[256];
  __shared__ uint32_t wc[RS_T / 64][256];
  rs_scatter(kin, vin, n, np, d, hist, tot, kout, vout, (int)blockIdx.x, run, wc);
}

// one radix pass of two sorts in each launch (sdx_group_step): partitions [0, a.np) sort a's keys,
// the rest b's
struct RsPass {
  const uint32_t* kin;
  const uint32_t* vin;
  uint32_t* kout;
  uint32_t* vout;
  uint32_t* hist;
  uint32_t* tot;
  int n, np;
};
__global__ __launch_bounds__(RS_T) void k_rs_hist2(RsPass a, RsPass b, int d) {
  __shared__ uint32_t c[256];
  const bool second = (int)blockIdx.x >= a.np;
  const RsPass& x = second ? b : a;
  rs_hist(x.kin, x.n, x.np, d, x.hist, second ? (int)blockIdx.x - a.np : (int)blockIdx.x, c);
}
__global__ __launch_bounds__(256) void k_rs_scan_rows2(RsPass a, RsPass b) {
  const bool second = blockIdx.x >= 256 / 4;
  const RsPass& x = second ? b : a;
  rs_scan_rows(x.hist, x.np, x.tot, (int)blockIdx.x - (second ? 256 / 4 : 0));
}
__global__ __launch_bounds__(RS_T) void k_rs_scatter2(RsPass a, RsPass b, int d) {
  __shared__ uint32_t run[256];
  __shared__ uint32_t wc[RS_T / 64][256];
  const bool second = (int)blockIdx.x >= a.np;
  const RsPass& x = second ? b : a;
  rs_scatter(x.kin, x.vin, x.n, x.np, d, x.hist, x.tot, x.kout, x.vout,
             second ? (int)blockIdx.x - a.np : (int)blockIdx.x, run, wc);
}

constexpr size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// workspace of the grouping: keys and message indices (two copies; the sorted indices end in the
// caller's order buffer) + the sort's counts
size_t group_bytes(int n) {
  if (n <= 0) return 0;
  const size_t np = (size_t)(n + RS_PART - 1) / RS_PART;
  return 4 * align256(4 * (size_t)n) + align256(4 * 256 * np) + align256(4 * 256);
}

// The grouped order of a batch's messages (or of its sel_dev subset): order[0, n) = message indices
// (the sel_dev of the k_pulses launch that follows).
bool group_messages(const void* bank_dev, int kind, const sdx_pulse_batch& b, int32_t* order, sdx_msg_rec* mrec,
                    uint8_t* work, size_t bytes, hipStream_t st) {
  const int n = b.sel_dev ? b.n_sel : b.n;
  const size_t need = group_bytes(n);
  if (!need || bytes < need) return false;
  const int np = (n + RS_PART - 1) / RS_PART;
  const size_t a = align256(4 * (size_t)n);
  uint32_t* k0 = reinterpret_cast<uint32_t*>(work);
  uint32_t* v0 = reinterpret_cast<uint32_t*>(work + a);
  uint32_t* k1 = reinterpret_cast<uint32_t*>(work + 2 * a);
  uint32_t* v1 = reinterpret_cast<uint32_t*>(work + 3 * a);
  uint32_t* hist = reinterpret_cast<uint32_t*>(work + 4 * a);
  uint32_t* tot = reinterpret_cast<uint32_t*>(work + 4 * a + align256(4 * 256 * (size_t)np));
  const int grid = (n + 255) / 256;
  if (kind == SDX_KIND_MU)
    hipLaunchKernelGGL((k_sig<SDX_KIND_MU>), dim3(grid), dim3(256), 0, st, bank_dev, b, k0, v0, mrec);
  else
    hipLaunchKernelGGL((k_sig<SDX_KIND_MS>), dim3(grid), dim3(256), 0, st, bank_dev, b, k0, v0, mrec);
  // the key's top RS_PASSES bytes (LSD order): (k0, v0) -> (k1, v1) -> (k0, v0) -> ..., the last
  // pass writing the message indices to order
  const int passes = kind == SDX_KIND_MU ? RS_PASSES : RS_PASSES_MS;
  for (int pi = 0; pi < passes; ++pi) {
    const int d = 4 - passes + pi;
    const bool even = (pi & 1) == 0;
    uint32_t* kin = even ? k0 : k1;
    uint32_t* vout = pi == passes - 1 ? reinterpret_cast<uint32_t*>(order) : (even ? v1 : v0);
    hipLaunchKernelGGL(k_rs_hist, dim3(np), dim3(RS_T), 0, st, kin, n, np, d, hist);
    hipLaunchKernelGGL(k_rs_scan_rows, dim3(256 / 4), dim3(256), 0, st, hist, np, tot);
    hipLaunchKernelGGL(k_rs_scatter, dim3(np), dim3(RS_T), 0, st, kin, even ? v0 : v1, n, np, d, hist, tot,
                       even ? k1 : k0, vout);
  }
  return hipGetLastError() == hipSuccess;
}

// The step's MU and MS groupings (same results as two group_messages calls) in 13 launches instead of
// 26: one k_sig2, then per radix pass one hist, one scan and one scatter launch over both sorts' partitions
bool group_messages2(const void* bank_dev, const sdx_pulse_batch& bmu, int32_t* omu, sdx_msg_rec* rmu, uint8_t* wmu,
                     size_t cmu, const sdx_pulse_batch& bms, int32_t* oms, sdx_msg_rec* rms, uint8_t* wms, size_t cms,
                     hipStream_t st) {
  static_assert(RS_PASSES == RS_PASSES_MS, "one pass count for both sorts");
  const int nmu = bmu.sel_dev ? bmu.n_sel : bmu.n, nms = bms.sel_dev ? bms.n_sel : bms.n;
  if (nmu <= 0 || nms <= 0 || cmu < group_bytes(nmu) || cms < group_bytes(nms)) return false;
  struct Side {
    uint32_t *k0, *v0, *k1, *v1, *hist, *tot;
    int n, np;
  };
  auto side = [](uint8_t* work, int n) {
    Side x;
    const size_t a = align256(4 * (size_t)n);
    x.n = n;
    x.np = (n + RS_PART - 1) / RS_PART;
    x.k0 = reinterpret_cast<uint32_t*>(work);
    x.v0 = reinterpret_cast<uint32_t*>(work + a);
    x.k1 = reinterpret_cast<uint32_t*>(work + 2 * a);
    x.v1 = reinterpret_cast<uint32_t*>(work + 3 * a);
    x.hist = reinterpret_cast<uint32_t*>(work + 4 * a);
    x.tot = reinterpret_cast<uint32_t*>(work + 4 * a + align256(4 * 256 * (size_t)x.np));
    return x;
  };
  const Side A = side(wmu, nmu), B = side(wms, nms);
  const int gmu = (nmu + 255) / 256, gms = (nms + 255) / 256;
  hipLaunchKernelGGL(k_sig2, dim3(gmu + gms), dim3(256), 0, st, bank_dev, SigSide{bmu, A.k0, A.v0, rmu},
                     SigSide{bms, B.k0, B.v0, rms}, gmu);
  for (int pi = 0; pi < RS_PASSES; ++pi) {
    const int d = 4 - RS_PASSES + pi;
    const bool even = (pi & 1) == 0;
    const bool last = pi == RS_PASSES - 1;
    auto pass = [&](const Side& x, int32_t* order) {
      return RsPass{even ? x.k0 : x.k1, even ? x.v0 : x.v1, even ? x.k1 : x.k0,
                    last ? reinterpret_cast<uint32_t*>(order) : (even ? x.v1 : x.v0), x.hist, x.tot, x.n, x.np};
    };
    const RsPass pa = pass(A, omu), pb = pass(B, oms);
    hipLaunchKernelGGL(k_rs_hist2, dim3(A.np + B.np), dim3(RS_T), 0, st, pa, pb, d);
    hipLaunchKernelGGL(k_rs_scan_rows2, dim3(2 * (256 / 4)), dim3(256), 0, st, pa, pb);
    hipLaunchKernelGGL(k_rs_scatter2, dim3(A.np + B.np), dim3(RS_T), 0, st, pa, pb, d);
  }
  return hipGetLastError() == hipSuccess;
}

}  // namespace sdx
