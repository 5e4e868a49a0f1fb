// sdx_mn.hip -- the MN (FSK) engine, hand-written HIP for gfx950.
//
// Lane = frame.  Per frame the kernel runs what MNParser.parse does after MN_PATTERN has matched
// (signalduino/parser/mn.py:79-191): for every 'modulation' protocol of the bank, in bank order,
//   the rfmode filter            (:83-93; folded into sdx_mn_batch.elig by the host),
//   length_in_range(len(hex))    (:95-101; helpers.py:124-166),
//   re.search(regexMatch, hex)   (:103-115; a search DFA of the bank blob, walked from HBM/L2),
//   the method                   (:117-173; helpers.py:223-716, restated on nibble values below),
//   payload = preamble + decoded (:121,155-166,176-177: no method -> the hex itself; a method's
//                                 empty list -> the string "[]", its first dict -> its payload).
// Method mode (sdx_mn_batch.method >= 1) runs one method alone: SDProtocols.ConvX(msg_data).
//
// Two passes over the frame, both in registers: pass 1 decides every (frame, protocol) outcome
// and its payload length; one wave-wide prefix sum and one atomic per wave reserve the records and
// the heap; pass 2 re-derives the outcomes and writes the records and the payload bytes of its
// frame into its own contiguous heap range with aligned 8-byte stores (W8).  The work is integer
// only (CRC/LFSR/XOR/popcount over <= 26 bytes, digit formatting): HBM-bound by design.
#include "sdx_device.h"

#include <string>

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
}

namespace sdxm {
using namespace sdx;

#define MD __device__ __forceinline__

// a hex digit's value; the contract is [0-9A-Fa-f] (the front end guarantees [0-9A-F])
MD uint32_t hv(uint8_t c) { return (uint32_t)((c & 15) + 9 * (c >> 6)); }
MD uint8_t hexch(uint32_t v) { return (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10); }
MD uint8_t upc(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

struct Frame {
  const uint8_t* s;
  int n;
  bool words;  // s is 4-byte aligned and readable in whole words (the frame's LDS slot)
  MD uint32_t byte(int k) const { return (hv(s[2 * k]) << 4) | hv(s[2 * k + 1]); }  // int(s[2k:2k+2], 16)
};

// the checksum tables, staged in LDS (bank.py mn_tables, include/sdx_bank.h SDX_MNTAB_*)
struct MnTab {
  const uint16_t* crc1021;
  const uint16_t* crc8005;
  const uint8_t* crc31;
  const uint16_t* lfsr8;   // [2 * 8][16]
  const uint16_t* lfsr21;  // [2 * 21][16]
};

// lfsr_digest16 (helpers.py:190-221) over bytes k0 .. k0+nb-1 of the frame, each XOR xr: the key
// sequence is data-independent, so the digest is the XOR of per-nibble table entries
MD uint32_t lfsr16(const Frame& f, int k0, int nb, const uint16_t* T, uint32_t xr) {
  uint32_t acc = 0;
  for (int k = 0; k < nb; ++k) {
    const uint32_t b = f.byte(k0 + k) ^ xr;
    acc ^= (uint32_t)T[32 * k + (b >> 4)] ^ (uint32_t)T[32 * k + 16 + (b & 15)];
  }
  return acc;
}

// _calc_crc16 (helpers.py:281-309) with init 0, no reflection, xorout 0 (both call sites), byte-wise
MD uint32_t crc16(const Frame& f, int k0, int nb, const uint16_t* T) {
  uint32_t crc = 0;
  for (int k = 0; k < nb; ++k) crc = ((crc << 8) & 0xFFFF) ^ (uint32_t)T[((crc >> 8) ^ f.byte(k0 + k)) & 0xFF];
  return crc;
}

MD int ndigits(uint32_t v) {
  int d = 1;
  while (v >= 10) {
    v /= 10;
    ++d;
  }
  return d;
}

// ---- sinks: Count (pass 1, lengths only) and W8 (pass 2, bytes) share one method body --------
struct Count {
  int n = 0;
  MD void put(uint8_t) { ++n; }
  MD void put_uint(uint32_t v) { n += ndigits(v); }
  MD void copy(const Frame&, int a, int e) { n += e - a; }
  MD void copy_xa(const Frame&, int a, int e) { n += e - a; }
  MD void copy_up(const Frame&, int a, int e) { n += e - a; }
};

// lane-private output: one 8-byte store per aligned word; the first and last words are written
// byte by byte, so no byte outside [dst, dst + n) is touched (neighbouring lanes' ranges abut)
struct W8 {
  uint8_t* w;
  uint64_t acc;
  int fill, head;
  MD explicit W8(uint8_t* dst)
      : w(dst - ((uintptr_t)dst & 7)), acc(0), fill((int)((uintptr_t)dst & 7)), head((int)((uintptr_t)dst & 7)) {}
  MD void flush_word() {
    if (head) {
      for (int k = head; k < 8; ++k) w[k] = (uint8_t)(acc >> (8 * k));
      head = 0;
    } else {
      *reinterpret_cast<uint64_t*>(w) = acc;
    }
    w += 8;
    acc = 0;
    fill = 0;
  }
  MD void put(uint8_t c) {
    acc |= (uint64_t)c << (8 * fill);
    if (++fill == 8) flush_word();
  }
  MD void put_uint(uint32_t v) {
    uint8_t t[10];
    int k = 0;
    do {
      t[k++] = (uint8_t)('0' + v % 10);
      v /= 10;
    } while (v);
    while (k) put(t[--k]);
  }
  // the low cnt (1..4) bytes of v
  MD void put4(uint32_t v, int cnt) {
    const uint64_t vv = cnt >= 4 ? (uint64_t)v : ((uint64_t)v & ((1ull << (8 * cnt)) - 1));
    const int f0 = fill;
    acc |= vv << (8 * f0);
    if (f0 + cnt < 8) {
      fill = f0 + cnt;
      return;
    }
    flush_word();
    acc = vv >> (8 * (8 - f0));  // f0 >= 4 here: shift 8..32
    fill = f0 + cnt - 8;
  }
  // a (the copy start) is a multiple of 4 at every call site, so LDS frames copy whole words
  MD void copy(const Frame& f, int a, int e) {
    if (f.words && !(a & 3)) {
      const uint32_t* w32 = reinterpret_cast<const uint32_t*>(f.s);
      for (int i = a; i < e; i += 4) put4(w32[i >> 2], e - i < 4 ? e - i : 4);
      return;
    }
    for (int i = a; i < e; ++i) put(f.s[i]);
  }
  MD void copy_xa(const Frame& f, int a, int e) {  // f"{int(c, 16) ^ 0xA:X}" per character
    if (f.words && !(a & 3)) {
      const uint32_t* w32 = reinterpret_cast<const uint32_t*>(f.s);
      for (int i = a; i < e; i += 4) {
        const uint32_t v = w32[i >> 2];
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) o |= (uint32_t)hexch(hv((uint8_t)(v >> (8 * k))) ^ 0xA) << (8 * k);
        put4(o, e - i < 4 ? e - i : 4);
      }
      return;
    }
    for (int i = a; i < e; ++i) put(hexch(hv(f.s[i]) ^ 0xA));
  }
  MD void copy_up(const Frame& f, int a, int e) {
    for (int i = a; i < e; ++i) put(upc(f.s[i]));
  }
  MD void finish() {
    for (int k = head; k < fill; ++k) w[k] = (uint8_t)(acc >> (8 * k));
  }
};

// one MN method on frame f: false = the method returns [] ; true = its payload went to out
template <class S>
MD bool run_method(int m, const Frame& f, S& out, const MnTab& tb) {
  const int n = f.n;
  switch (m) {
    case SDX_MN_LIGHTNING: {  // helpers.py:223-280: XOR 0xA, LFSR-16 gen 8810 key ABF9 over bytes 2..9
      if (n < 20) return false;
      const uint32_t chk = lfsr16(f, 2, 8, tb.lfsr8, 0xAA) ^ (((f.byte(0) ^ 0xAA) << 8) | (f.byte(1) ^ 0xAA));
      if (chk != 0x899E) return false;
      out.copy_xa(f, 0, 20);
      return true;
    }
    case SDX_MN_5IN1: {  // helpers.py:382-425: bytes 13..25 invert 0..12, popcount of 14..25 = byte 13
      if (n < 52) return false;
      uint32_t bits = 0, ref = 0;
      for (int i = 0; i < 13; ++i) {
        const uint32_t a = f.byte(i), inv = f.byte(i + 13);
        if ((a ^ inv) != 0xFF) return false;
        if (i == 0) ref = inv;
        else bits += __popc(inv);
      }
      if (bits != ref) return false;
      out.copy(f, 28, 52);
      return true;
    }
    case SDX_MN_6IN1: {  // helpers.py:427-471: CRC-16/XMODEM of bytes 2..16 = bytes 0..1, sum 2..17 = 0xFF
      if (n < 36) return false;
      if (crc16(f, 2, 15, tb.crc1021) != ((f.byte(0) << 8) | f.byte(1))) return false;
      uint32_t sum = 0;
      for (int i = 2; i < 18; ++i) sum += f.byte(i);
      if ((sum & 0xFF) != 0xFF) return false;
      out.copy(f, 0, n);
      return true;
    }
    case SDX_MN_7IN1: {  // helpers.py:473-523: byte 21 != '00', XOR 0xA, LFSR-16 gen 8810 key BA95
      if (n < 46) return false;
      if (f.s[42] == '0' && f.s[43] == '0') return false;
      const uint32_t chk = lfsr16(f, 2, 21, tb.lfsr21, 0xAA) ^ (((f.byte(0) ^ 0xAA) << 8) | (f.byte(1) ^ 0xAA));
      if (chk != 0x6DF1) return false;
      out.copy_xa(f, 0, n);
      return true;
    }
    case SDX_MN_PCA301: {  // helpers.py:525-579: CRC-16 poly 8005 of bytes 0..9 = bytes 10..11
      if (n < 24) return false;
      if (crc16(f, 0, 10, tb.crc8005) != ((f.byte(10) << 8) | f.byte(11))) return false;
      const char* hdr = "OK 24";
      for (int i = 0; i < 5; ++i) out.put((uint8_t)hdr[i]);
      for (int i = 0; i < 10; ++i) {
        out.put(' ');
        out.put_uint(i == 5 ? (f.byte(5) & 0x0F) : f.byte(i));
      }
      out.put(' ');
      out.copy_up(f, 20, 24);
      return true;
    }
    case SDX_MN_KOPP: {  // helpers.py:581-628: XOR 0xAA over byte0 + 1 bytes = the next byte
      if (n < 4) return false;
      const int anz = (int)f.byte(0) + 1;
      if (n < 2 * anz + 2) return false;
      uint32_t acc = 0xAA;
      for (int i = 0; i < anz; ++i) acc ^= f.byte(i);
      if (acc != f.byte(anz)) return false;
      out.put('k');
      out.put('r');
      out.copy(f, 0, 2 * anz);
      return true;
    }
    case SDX_MN_LACROSSE: {  // helpers.py:630-716: CRC-8 poly 31 (MSB first) of bytes 0..3 = byte 4
      if (n < 10) return false;
      uint32_t crc = 0;
      for (int i = 0; i < 4; ++i) crc = tb.crc31[crc ^ f.byte(i)];
      if (crc != f.byte(4)) return false;
      const uint32_t b0 = f.byte(0), b1 = f.byte(1), b2 = f.byte(2), b3 = f.byte(3);
      const uint32_t addr = ((b0 & 0x0F) << 2) | ((b1 & 0xC0) >> 6);
      const int traw = (int)((b1 & 0x0F) * 100 + ((b2 & 0xF0) >> 4) * 10 + (b2 & 0x0F));
      const double t = (double)traw / 10.0 - 40.0;  // fp64 like Python (-ffp-contract=off)
      if (t >= 60.0 || t <= -40.0) return false;
      const uint32_t sensor = (b3 & 0x7F) == 125 ? 2u : 1u;
      const uint32_t scaled = (uint32_t)(int)(t * 10.0 + 1000.0) & 0xFFFF;  // int() truncates (> 0 here)
      const char* hdr = "OK 9";
      for (int i = 0; i < 4; ++i) out.put((uint8_t)hdr[i]);
      const uint32_t v[5] = {addr, sensor | ((b1 & 0x20) << 2), (scaled >> 8) & 0xFF, scaled & 0xFF, b3};
      for (int i = 0; i < 5; ++i) {
        out.put(' ');
        out.put_uint(v[i]);
      }
      return true;
    }
  }
  return false;
}

constexpr int MN_THREADS = 256;
constexpr int MN_SLOT = 128;               // frames of <= 128 hex characters are staged in LDS
constexpr int MN_SLOT_W = MN_SLOT / 4 + 1;  // words per lane slot (odd stride: fewer bank conflicts)

// per-frame caches of the two per-frame facts several protocols share: regexMatch outcomes (by
// distinct pattern, sdx_mn_proto.dfa_slot) and method outcomes + decoded lengths (by method)
struct MnCache {
  uint32_t dfa_done = 0, dfa_ok = 0;
  uint32_t m_done = 0, m_ok = 0;
  uint64_t len_lo = 0, len_hi = 0;  // 16-bit decoded length of method m: bits 16 * (m & 3) of lo (m < 4) / hi
  MD int len(int m) const { return (int)(((m < 4 ? len_lo : len_hi) >> (16 * (m & 3))) & 0xFFFF); }
  MD void set_len(int m, int v) {
    if (m < 4) len_lo |= (uint64_t)(v & 0xFFFF) << (16 * (m & 3));
    else len_hi |= (uint64_t)(v & 0xFFFF) << (16 * (m & 3));
  }
};

// parser-mode outcome of protocol p on frame f: -1 no result, else the payload length
MD int mn_outcome(const BankView& bv, const sdx_mn_proto* r, const Frame& f, MnCache& c, const MnTab& tb) {
  const int lmin = cld(&r->lir_min), lmax = cld(&r->lir_max);
  if ((lmin != -1 && f.n < lmin) || f.n > lmax) return -1;
  const int d = cld(&r->dfa);
  if (d >= 0) {
    const int slot = cld(&r->dfa_slot);
    if (!((c.dfa_done >> slot) & 1u)) {
      c.dfa_done |= 1u << slot;
      if (dfa_accepts(bv, d, cld(&bv.dfa[d].start), f.s, f.n)) c.dfa_ok |= 1u << slot;
    }
    if (!((c.dfa_ok >> slot) & 1u)) return -1;
  }
  const int m = cld(&r->method);  // wave-uniform
  if (m == SDX_MN_MISSING) return -1;
  const int pre = cld(&r->pre_len);
  if (m == SDX_MN_RAW) return pre + f.n;
  if (!((c.m_done >> m) & 1u)) {
    c.m_done |= 1u << m;
    Count cnt;
    if (run_method(m, f, cnt, tb)) {
      c.m_ok |= 1u << m;
      c.set_len(m, cnt.n);
    }
  }
  return pre + (((c.m_ok >> m) & 1u) ? c.len(m) : 2);
}

__global__ __launch_bounds__(MN_THREADS) void k_mn(const void* __restrict__ bank, sdx_mn_batch b, sdx_out out) {
  __shared__ uint32_t slots[MN_THREADS / 64][64][MN_SLOT_W];
  __shared__ uint4 tabs[(SDX_MNTAB_BYTES + 15) / 16];
  const BankView bv = bank_view(bank);
  {  // checksum tables -> LDS (3 KB, one 16-byte load per thread)
    const uint4* src = reinterpret_cast<const uint4*>(bv.base + bv.hdr->off_mntab);
    for (int i = threadIdx.x; i < (SDX_MNTAB_BYTES + 15) / 16; i += MN_THREADS) tabs[i] = src[i];
    __syncthreads();
  }
  const uint8_t* tb8 = reinterpret_cast<const uint8_t*>(tabs);
  const MnTab tb{reinterpret_cast<const uint16_t*>(tb8 + SDX_MNTAB_CRC1021),
                 reinterpret_cast<const uint16_t*>(tb8 + SDX_MNTAB_CRC8005), tb8 + SDX_MNTAB_CRC31,
                 reinterpret_cast<const uint16_t*>(tb8 + SDX_MNTAB_LFSR8),
                 reinterpret_cast<const uint16_t*>(tb8 + SDX_MNTAB_LFSR21)};
  const sdx_mn_proto* mn = uniform_ptr((const sdx_mn_proto*)(bv.base + bv.hdr->off_mn));
  const int nmn = (int)bv.hdr->n_mn;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntot = b.sel_dev ? b.n_sel : b.n;
  const int gi = blockIdx.x * MN_THREADS + threadIdx.x;
  const bool valid = gi < ntot;
  const int msg = valid ? (b.sel_dev ? b.sel_dev[gi] : gi) : 0;
  int64_t off = 0;
  int n = 0;
  if (valid) {
    off = b.offsets_dev[msg];
    n = b.len_dev ? b.len_dev[msg] : (int)(b.offsets_dev[msg + 1] - off);
  }
  // ---- stage the wave's short frames into the lanes' LDS slots: one frame at a time, every lane
  // copies one realigned 4-byte word (sdx_mn_batch contract: hex_dev readable 8 bytes past a frame)
  // batches of 8 frames: the 8 loads are issued back to back, then stored (latencies overlap)
  const bool stage_me = valid && n <= MN_SLOT && n > 0;
  const uint64_t sm = __ballot(stage_me);
  for (int j0 = 0; j0 < 64; j0 += 8) {
    if (!((sm >> j0) & 0xFFull)) continue;  // uniform
    uint32_t v[8];
    uint32_t stm = 0;  // bit u: this lane stores a word of frame j0 + u
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u;
      const int lo = __shfl((int)(uint32_t)off, j), hi = __shfl((int)(uint32_t)((uint64_t)off >> 32), j);
      const int64_t o = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
      const int nj = __shfl(n, j);
      const int sh = (int)(((uintptr_t)b.hex_dev + o) & 3);
      const uint32_t* sw = reinterpret_cast<const uint32_t*>(b.hex_dev + o - sh);
      v[u] = 0;
      if (((sm >> j) & 1ull) && lane < ((nj + 3) >> 2)) {
        v[u] = __builtin_amdgcn_alignbyte(sw[lane + 1], sw[lane], sh);
        stm |= 1u << u;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if ((stm >> u) & 1u) slots[wave][j0 + u][lane] = v[u];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  Frame f{b.hex_dev + off, n, false};
  if (valid && n <= MN_SLOT) {
    f.s = reinterpret_cast<const uint8_t*>(&slots[wave][lane][0]);
    f.words = true;
  }
  // ---- pass 1: outcomes and sizes
  uint64_t hit = 0;
  int nrec = 0, nbytes = 0;
  MnCache cache;
  if (b.method >= 0) {
    Count c;
    if (valid && run_method(b.method, f, c, tb)) {
      hit = 1;
      nrec = 1;
      nbytes = c.n;
    }
  } else {
    for (int p = 0; p < nmn; ++p) {
      if (!((b.elig >> p) & 1)) continue;  // uniform
      const int len = valid ? mn_outcome(bv, mn + p, f, cache, tb) : -1;
      if (len >= 0) {
        hit |= 1ull << p;
        ++nrec;
        nbytes += len;
      }
    }
  }
  // ---- reserve: wave prefix sums, one atomic per wave and buffer
  int ir = nrec, ib = nbytes;
  for (int d = 1; d < WAVE; d <<= 1) {
    const int tr = __shfl_up(ir, d), tb = __shfl_up(ib, d);
    if (lane >= d) {
      ir += tr;
      ib += tb;
    }
  }
  const int wrec = __shfl(ir, WAVE - 1), wbytes = __shfl(ib, WAVE - 1);
  uint32_t rbase = 0, hbase = 0;
  int st = 0;
  if (lane == 0 && wrec) {
    rbase = atomicAdd(&out.cursor_dev[0], (uint32_t)wrec);
    hbase = atomicAdd(&out.cursor_dev[1], (uint32_t)wbytes);
    if ((uint64_t)rbase + wrec > out.rec_cap || (uint64_t)hbase + wbytes > out.heap_cap) {
      st = 3;
      atomicOr(&out.cursor_dev[2], 1u);
    }
  }
  rbase = (uint32_t)__shfl((int)rbase, 0);
  hbase = (uint32_t)__shfl((int)hbase, 0);
  st = __shfl(st, 0);
  if (!valid) return;
  const uint32_t r0 = rbase + (uint32_t)(ir - nrec);
  sdx_desc dsc;
  dsc.rec_begin = r0;
  dsc.raise_kind = 0;
  if (st) {
    dsc.status = SDX_ST_OVF_OUT;
    dsc.n_rec = 0;
    out.desc_dev[msg] = dsc;
    return;
  }
  dsc.status = SDX_ST_OK;
  dsc.n_rec = (uint16_t)nrec;
  out.desc_dev[msg] = dsc;
  if (!nrec) return;
  // ---- pass 2: records + payload bytes into [hbase + ib - nbytes, +nbytes)
  uint32_t h = hbase + (uint32_t)(ib - nbytes);
  W8 w(out.heap_dev + h);
  uint32_t q = r0;
  if (b.method >= 0) {
    const int len0 = nbytes;
    run_method(b.method, f, w, tb);
    sdx_result o;
    o.payload_off = h;
    o.payload_len = (uint16_t)len0;
    o.proto = (uint16_t)b.method;
    o.bit_length = 0;
    o.msg = (uint32_t)msg;
    out.rec_dev[q] = o;
  } else {
    uint64_t hm = hit;
    while (hm) {
      const int p = __builtin_ctzll(hm);
      hm &= hm - 1;
      const sdx_mn_proto* r = mn + p;
      const int pre = r->pre_len, m = r->method;
      const uint8_t* ps = bv.str + r->pre_off;
      for (int i = 0; i < pre; ++i) w.put(ps[i]);
      int len = pre;
      if (m == SDX_MN_RAW) {
        w.copy(f, 0, f.n);
        len += f.n;
      } else {
        if ((cache.m_ok >> m) & 1u) {  // pass 1 ran this method on this frame
          run_method(m, f, w, tb);
          len += cache.len(m);
        } else {  // str([]) (mn.py:164-166)
          w.put('[');
          w.put(']');
          len += 2;
        }
      }
      sdx_result o;
      o.payload_off = h;
      o.payload_len = (uint16_t)len;
      o.proto = (uint16_t)p;
      o.bit_length = 0;
      o.msg = (uint32_t)msg;
      out.rec_dev[q++] = o;
      h += (uint32_t)len;
    }
  }
  w.finish();
}

}  // namespace sdxm

namespace sdx {  // sdx_kernels.hip
const void* bank_dev_ptr(const sdx_bank* b);
const sdx_bank_hdr* bank_hdr(const sdx_bank* b);
}  // namespace sdx

extern "C" int sdx_demod_mn(const sdx_bank* bank, const sdx_mn_batch* batch, const sdx_out* out, void* hip_stream) {
  if (!bank || !batch || !out) return sdx::set_error(SDX_EINVAL, "sdx_demod_mn: null argument");
  if (batch->method != -1 && (batch->method < SDX_MN_LIGHTNING || batch->method > SDX_MN_LACROSSE))
    return sdx::set_error(SDX_EINVAL, "sdx_demod_mn: method must be -1 (parser mode) or an sdx_mn_method");
  if (sdx::bank_hdr(bank)->n_mn > SDX_MN_MAX) return sdx::set_error(SDX_EBANK, "sdx_demod_mn: too many MN protocols");
  const int ntot = batch->sel_dev ? batch->n_sel : batch->n;
  if (ntot <= 0) return SDX_OK;
  const int grid = (ntot + sdxm::MN_THREADS - 1) / sdxm::MN_THREADS;
  hipLaunchKernelGGL(sdxm::k_mn, dim3(grid), dim3(sdxm::MN_THREADS), 0, (hipStream_t)hip_stream,
                     sdx::bank_dev_ptr(bank), *batch, *out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_demod_mn: ") + hipGetErrorString(e));
  return SDX_OK;
}
