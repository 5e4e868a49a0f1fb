// sdx_units.hip -- the unit-level entry (sdx_units): one reference helper function evaluated on n
// independent inputs, lane = item, hand-written HIP for gfx950.
//
// These are the functions the reference's SDProtocols class exposes besides demodulate*, and that
// its own unit tests call directly (tests/test_postdemodulation.py, test_manchester_protocols.py,
// test_pattern_utils.py, test_helpers.py).  The drop-in SDProtocols (pysignalduino_amd/units.py)
// binds them as thin wrappers over this launch; the device code is the same that the MU/MS/MC
// kernels run (sdx_device.h pd_*, sdx_mc.h mc_method), plus pattern_exists on arbitrary fp64
// inputs (pattern_utils.py:34-136) and the hex/bit helpers (helpers.py:6-64, 168-188).
//
// Per item i: desc[i] = {rec_begin = i, n_rec = 1, status OK | RAISED(kind)}, rec[i] = {payload at
// heap[out_off[i] ..], payload_len, proto = 0 (a value was returned, the payload holds it) or an
// op-specific failure code, bit_length = op-specific aux, msg = i}.  No atomics, no ordering: the
// host sized every item's output range.
#include "sdx_mc.h"

#include <string>

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
}

namespace sdxu {
using namespace sdx;

#define UD __device__ __forceinline__

UD uint8_t hexch(int v) { return (uint8_t)(v < 10 ? '0' + v : 'A' + v - 10); }
UD int hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return -1;
}

struct UnitRes {
  int len;     // payload bytes written
  int code;    // 0 = value returned (payload), > 0 = op-specific failure
  int aux;
  int raise;   // enum sdx_raise
};

// ---- postDemo_* (postdemodulation.py:27-730) on bits 0/1 -------------------------------------
UD UnitRes u_postdemo(int which, const uint8_t* in, int n, uint8_t* out) {
  int no = 0;
  const int rc = run_postdemo(which, in, n, out, &no);
  if (rc < 0) return UnitRes{0, 0, 0, SDX_RAISE_VALUE};
  if (rc == 0) return UnitRes{0, 1, 0, 0};  // (0, None)
  return UnitRes{no, 0, 0, 0};
}

// ---- hex_to_bin_str (helpers.py:168-188), after the optional polarity translate of
// _convert_mc_hex_to_bits (manchester.py:33-36: uppercase digits only).  code 1 = None.
UD UnitRes u_hex2bin(const uint8_t* in, int n, int invert, uint8_t* out) {
  if (n <= 0) return UnitRes{0, 1, 0, 0};  // int('', 16) -> ValueError -> None
  for (int i = 0; i < n; ++i)
    if (hexv(in[i]) < 0) return UnitRes{0, 1, 0, 0};
  int q = 0;
  bool started = false;
  for (int i = 0; i < n; ++i) {
    const uint8_t c = in[i];
    int v = hexv(c);
    if (invert && !(c >= 'a' && c <= 'f')) v = 15 - v;
    if (!v && !started && i != n - 1) continue;  // bin(int(h, 16)) drops leading zero nibbles
    started = true;
    for (int b = 3; b >= 0; --b) out[q++] = (uint8_t)('0' + ((v >> b) & 1));
  }
  return UnitRes{q, 0, 0, 0};
}

// ---- bin_str_2_hex_str (helpers.py:28-64): code 1 = None (a character other than '0'/'1')
UD UnitRes u_bin2hex(const uint8_t* in, int n, uint8_t* out) {
  for (int i = 0; i < n; ++i)
    if (in[i] != '0' && in[i] != '1') return UnitRes{0, 1, 0, 0};
  const int nd = (n + 3) >> 2;
  for (int d = 0; d < nd; ++d) {
    const int de = n - 4 * (nd - 1 - d), da = de - 4 > 0 ? de - 4 : 0;
    int v = 0;
    for (int i = da; i < de; ++i) v = (v << 1) | (in[i] - '0');
    out[d] = hexch(v);
  }
  return UnitRes{nd, 0, 0, 0};
}

// ---- mc2dmc (helpers.py:6-26) on any ASCII string: E = s.replace('1','lh').replace('0','hl'),
// then '0' if E[i] == E[i+1] else '1' for i = 1, 3, ... < len(E) - 1
UD UnitRes u_mc2dmc(const uint8_t* in, int n, uint8_t* out) {
  // E as a stream: character k of s expands to 1 or 2 characters
  int q = 0, pos = 0;
  uint8_t prev = 0;  // E[pos - 1]
  int elen = 0;
  for (int k = 0; k < n; ++k) elen += (in[k] == '0' || in[k] == '1') ? 2 : 1;
  for (int k = 0; k < n; ++k) {
    const uint8_t c = in[k];
    uint8_t e[2];
    int m = 1;
    if (c == '1') { e[0] = 'l'; e[1] = 'h'; m = 2; }
    else if (c == '0') { e[0] = 'h'; e[1] = 'l'; m = 2; }
    else e[0] = c;
    for (int j = 0; j < m; ++j, ++pos) {
      // pair (pos - 1, pos) with pos - 1 odd and pos - 1 < len(E) - 1
      if (pos >= 2 && ((pos - 1) & 1) && pos - 1 < elen - 1) out[q++] = (prev == e[j]) ? '0' : '1';
      prev = e[j];
    }
  }
  return UnitRes{q, 0, 0, 0};
}

// ---- pattern_exists (pattern_utils.py:34-136) on arbitrary fp64 values --------------------------
// item bytes: [npat][len_0 .. len_{npat-1}][id bytes][raw_data]; values: nsearch search values then
// npat pattern values (dict order).  code 1 = -1.
constexpr int PX_MAXS = 32, PX_MAXP = 16;

UD double calc_tol(double v) {  // calculate_tolerance (:15-26)
  const double a = fabs(v);
  if (a > 3.0) return a > 16.0 ? a * 0.18 : a * 0.3;
  return 1.0;
}

UD UnitRes u_pexists(const uint8_t* in, int nin, const double* val, int nsearch, uint8_t* out) {
  const int npat = in[0];
  int idoff[PX_MAXP], idlen[PX_MAXP];
  int off = 1 + npat;
  for (int k = 0; k < npat; ++k) {
    idlen[k] = in[1 + k];
    idoff[k] = off;
    off += idlen[k];
  }
  const uint8_t* raw = in + off;
  const int nraw = nin - off;
  const double* sv = val;
  const double* pv = val + nsearch;
  // unique search values in first-appearance order (set membership: fp64 ==)
  double uv[PX_MAXS];
  int umap[PX_MAXS];
  int nu = 0;
  for (int s = 0; s < nsearch; ++s) {
    int u = -1;
    for (int t = 0; t < nu; ++t)
      if (uv[t] == sv[s]) { u = t; break; }
    if (u < 0) { u = nu; uv[nu++] = sv[s]; }
    umap[s] = u;
  }
  // candidates per unique value: gap <= 0.001 or gap <= tol, stable-sorted by gap
  uint8_t cand[PX_MAXS][PX_MAXP];
  int cnt[PX_MAXS];
  long long total = 1;
  for (int u = 0; u < nu; ++u) {
    const double tol = calc_tol(uv[u]);
    double gap[PX_MAXP];
    int c = 0;
    for (int k = 0; k < npat; ++k) {
      const double g = fabs(pv[k] - uv[u]);
      if (g <= 0.001 || g <= tol) {
        int j = c++;  // insertion sort, stable: move past strictly larger gaps only
        while (j > 0 && gap[j - 1] > g) { gap[j] = gap[j - 1]; cand[u][j] = cand[u][j - 1]; --j; }
        gap[j] = g;
        cand[u][j] = (uint8_t)k;
      }
    }
    if (c == 0) return UnitRes{0, 1, 0, 0};
    cnt[u] = c;
    total *= c;
    if (total > 10000) total = 10001;
  }
  if (total > 10000) return UnitRes{0, 1, 0, 0};
  int digit[PX_MAXS];
  for (int u = 0; u < nu; ++u) digit[u] = 0;
  for (long long it = 0; it < total; ++it) {
    uint32_t used = 0;
    bool dup = false;
    for (int u = 0; u < nu; ++u) {
      const int k = cand[u][digit[u]];
      if (used & (1u << k)) dup = true;
      used |= 1u << k;
    }
    if (!dup) {
      int tlen = 0;
      for (int s = 0; s < nsearch; ++s) tlen += idlen[cand[umap[s]][digit[umap[s]]]];
      for (int p = 0; p + tlen <= nraw; ++p) {  // target in raw_data
        bool ok = true;
        int q = p;
        for (int s = 0; s < nsearch && ok; ++s) {
          const int k = cand[umap[s]][digit[umap[s]]];
          for (int j = 0; j < idlen[k]; ++j, ++q)
            if (raw[q] != in[idoff[k] + j]) { ok = false; break; }
        }
        if (ok) {
          int w = 0;
          for (int s = 0; s < nsearch; ++s) {
            const int k = cand[umap[s]][digit[umap[s]]];
            for (int j = 0; j < idlen[k]; ++j) out[w++] = in[idoff[k] + j];
          }
          return UnitRes{w, 0, 0, 0};
        }
      }
    }
    for (int u = nu - 1; u >= 0; --u) {  // itertools.product: the last list varies fastest
      if (digit[u] + 1 < cnt[u]) { digit[u]++; break; }
      digit[u] = 0;
    }
  }
  return UnitRes{0, 1, 0, 0};
}

// ---- MC methods (manchester.py:207-795, helpers.py:90-122) on a '0'/'1' string ------------------
constexpr int UNIT_THREADS = 256;

__global__ __launch_bounds__(UNIT_THREADS) void k_units(sdx_unit_batch b, sdx_out out) {
  __shared__ uint64_t bits[MC_MAXW * UNIT_THREADS];  // lane-strided words (LaneBits layout)
  const int tid = threadIdx.x;
  const int i = blockIdx.x * UNIT_THREADS + tid;
  if (i >= b.n) return;
  const int64_t o0 = b.in_off_dev[i];
  const int n = (int)(b.in_off_dev[i + 1] - o0);
  const uint8_t* in = b.in_dev + o0;
  const int arg = b.arg_dev ? b.arg_dev[i] : 0;
  const int64_t w0 = b.out_off_dev[i];
  uint8_t* dst = out.heap_dev + w0;
  UnitRes r{0, 0, 0, 0};
  switch (b.op) {
    case SDX_UNIT_POSTDEMO: r = u_postdemo(arg, in, n, dst); break;
    case SDX_UNIT_HEX2BIN: r = u_hex2bin(in, n, arg, dst); break;
    case SDX_UNIT_BIN2HEX: r = u_bin2hex(in, n, dst); break;
    case SDX_UNIT_MC2DMC: r = u_mc2dmc(in, n, dst); break;
    case SDX_UNIT_PEXISTS: {
      const int64_t v0 = b.val_off_dev[i];
      if (n < 1 || in[0] > PX_MAXP || arg < 0 || arg > PX_MAXS) { r.raise = SDX_RAISE_TYPE; break; }  // host contract
      r = u_pexists(in, n, b.val_dev + v0, arg, dst);
      break;
    }
    case SDX_UNIT_MC_METHOD: {
      const sdx_mc_proto* rec = reinterpret_cast<const sdx_mc_proto*>(b.mcrec_dev) + i;
      if (n > MC_MAXW * 64) { r.raise = SDX_RAISE_TYPE; break; }  // host contract (SDX_UNIT_MC_BITS)
      for (int w = 0; w < MC_MAXW; ++w) bits[w * UNIT_THREADS + tid] = 0;
      for (int k = 0; k < n; ++k)
        if (in[k] == '1') bits[(k >> 6) * UNIT_THREADS + tid] |= 1ull << (63 - (k & 63));
      const LaneBits B{&bits[tid], MC_MAXW, false}, D{&bits[tid], MC_MAXW, true};
      const McOut o = mc_method(rec, rec->method, B, n, arg, D);
      if (o.rc == -1) r.raise = SDX_RAISE_TYPE;
      else if (o.rc == -2) r.raise = SDX_RAISE_VALUE;
      else if (o.rc == 0) { r.code = o.why; r.aux = o.aux; }
      else {
        mc_write(rec, o, B, n, arg, dst);
        r.len = o.len;
        r.aux = o.kind;
      }
      break;
    }
    default: r.raise = SDX_RAISE_TYPE;
  }
  sdx_desc d;
  d.rec_begin = (uint32_t)i;
  d.n_rec = r.raise ? 0 : 1;
  d.status = r.raise ? SDX_ST_RAISED : SDX_ST_OK;
  d.raise_kind = (uint8_t)r.raise;
  out.desc_dev[i] = d;
  sdx_result res;
  res.payload_off = (uint32_t)w0;
  res.payload_len = (uint16_t)r.len;
  res.proto = (uint16_t)r.code;
  res.bit_length = (uint32_t)r.aux;
  res.msg = (uint32_t)i;
  out.rec_dev[i] = res;
}

}  // namespace sdxu

extern "C" int sdx_units(const sdx_unit_batch* batch, const sdx_out* out, void* hip_stream) {
  if (!batch || !out) return sdx::set_error(SDX_EINVAL, "null argument");
  if (batch->n <= 0) return SDX_OK;
  if (!batch->in_dev || !batch->in_off_dev || !batch->out_off_dev || !out->desc_dev || !out->rec_dev ||
      !out->heap_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_units: missing buffer");
  if (batch->op == SDX_UNIT_PEXISTS && (!batch->val_dev || !batch->val_off_dev))
    return sdx::set_error(SDX_EINVAL, "sdx_units: pattern_exists needs val_dev / val_off_dev");
  if (batch->op == SDX_UNIT_MC_METHOD && !batch->mcrec_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_units: MC methods need mcrec_dev");
  if (batch->op < SDX_UNIT_POSTDEMO || batch->op > SDX_UNIT_MC_METHOD)
    return sdx::set_error(SDX_EINVAL, "sdx_units: unknown op");
  if ((uint32_t)batch->n > out->rec_cap) return sdx::set_error(SDX_EINVAL, "sdx_units: rec_cap < n");
  const int grid = (batch->n + sdxu::UNIT_THREADS - 1) / sdxu::UNIT_THREADS;
  hipLaunchKernelGGL(sdxu::k_units, dim3(grid), dim3(sdxu::UNIT_THREADS), 0, (hipStream_t)hip_stream, *batch, *out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("k_units: ") + hipGetErrorString(e));
  return SDX_OK;
}
