// sdx_json.hip -- publish-ready JSON of decoded messages, hand-written HIP for gfx950.
//
// MqttPublisher._message_to_json (signalduino/mqtt.py:227-245) is json.dumps(d, indent=4) of
//   d = {"protocol_id": str, "payload": str, "metadata": dict}     (asdict(message) minus "raw")
// with Python's defaults: ", " / ": " separators broken into lines by indent=4, ensure_ascii
// escapes (\" \\ \n \r \t \b \f, \u00XX for other control and all non-ASCII characters, lower-case
// hex), float.__repr__ and null for None.  The metadata dict of each kind is fixed by the
// demodulators (message_unsynced.py:282-290, message_synced.py:233-241, sd_protocols.py:102-109 +
// manchester.py:136-140, parser/mn.py:181-191), so the texts are built here from fragments:
// protocol strings pre-rendered by Python's json on the host (bank.py, sdx_json_rec), the payload
// bytes of the demodulation launch, and the per-line fields of the front end.  The only floats the
// device prints are integral or half-integral values below 1e15 (abs(P[CP]), calc_rssi,
// round(..., 0)), whose repr is "<integer>.0" / "<integer>.5".
//
// Lane = published item (a line's first result, or one result record).  Pass 1 sizes the text
// (Count sink), one wave prefix sum + one atomic reserve the bytes, pass 2 writes them (J8 sink,
// aligned 8-byte stores into the lane's own range).
#include "sdx_device.h"

#include <string>

namespace sdx {  // sdx_kernels.hip
int set_error(int code, const std::string& msg);
const void* bank_dev_ptr(const sdx_bank* b);
}  // namespace sdx

namespace sdxj {
using namespace sdx;

#define JD __device__ __forceinline__

JD int ndig64(uint64_t v) {
  int d = 1;
  while (v >= 10) {
    v /= 10;
    ++d;
  }
  return d;
}

// bytes json.dumps(ensure_ascii=True) needs for one character of a str
JD int esc_len(uint8_t c) {
  if (c == '"' || c == '\\' || c == '\n' || c == '\r' || c == '\t' || c == '\b' || c == '\f') return 2;
  if (c < 0x20 || c >= 0x80) return 6;
  return 1;
}

struct Count {
  uint32_t n = 0;
  JD void put(uint8_t) { ++n; }
  JD void lit(const char* s) {
    while (*s) {
      ++n;
      ++s;
    }
  }
  JD void bytes(const uint8_t* p, int k) { n += (uint32_t)k; }
  JD void esc(const uint8_t* p, int k) {
    for (int i = 0; i < k; ++i) n += (uint32_t)esc_len(p[i]);
  }
  JD void u64(uint64_t v) { n += (uint32_t)ndig64(v); }
};

struct J8 {
  uint8_t* w;
  uint64_t acc;
  int fill, head;
  JD explicit J8(uint8_t* dst)
      : w(dst - ((uintptr_t)dst & 7)), acc(0), fill((int)((uintptr_t)dst & 7)), head((int)((uintptr_t)dst & 7)) {}
  JD void flush_word() {
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
  JD void put(uint8_t c) {
    acc |= (uint64_t)c << (8 * fill);
    if (++fill == 8) flush_word();
  }
  JD void lit(const char* s) {
    while (*s) put((uint8_t)*s++);
  }
  JD void bytes(const uint8_t* p, int k) {
    for (int i = 0; i < k; ++i) put(p[i]);
  }
  JD void esc(const uint8_t* p, int k) {
    const char* hx = "0123456789abcdef";
    for (int i = 0; i < k; ++i) {
      const uint8_t c = p[i];
      switch (c) {
        case '"': put('\\'); put('"'); break;
        case '\\': put('\\'); put('\\'); break;
        case '\n': put('\\'); put('n'); break;
        case '\r': put('\\'); put('r'); break;
        case '\t': put('\\'); put('t'); break;
        case '\b': put('\\'); put('b'); break;
        case '\f': put('\\'); put('f'); break;
        default:
          if (c < 0x20 || c >= 0x80) {
            put('\\'); put('u'); put('0'); put('0');
            put((uint8_t)hx[c >> 4]);
            put((uint8_t)hx[c & 15]);
          } else {
            put(c);
          }
      }
    }
  }
  JD void u64(uint64_t v) {
    uint8_t t[20];
    int k = 0;
    do {
      t[k++] = (uint8_t)('0' + v % 10);
      v /= 10;
    } while (v);
    while (k) put(t[--k]);
  }
  JD void finish() {
    for (int k = head; k < fill; ++k) w[k] = (uint8_t)(acc >> (8 * k));
  }
};

// repr(float) of a half-integral value 2x = v2 (|x| < 1e15): "<int>.0" or "<int>.5"
template <class S>
JD void half_float(S& o, int64_t v2, bool neg_zero) {
  if (v2 < 0 || neg_zero) o.put('-');
  const uint64_t a = (uint64_t)(v2 < 0 ? -v2 : v2);
  o.u64(a >> 1);
  o.put('.');
  o.put((a & 1) ? '5' : '0');
}

// raw meta string (meta_dev: 15 bytes, length at byte 15, 255 = absent)
struct Raw {
  const uint8_t* p;
  int n;  // -1 = None
};
JD Raw meta_str(const uint8_t* m) { return Raw{m, m[15] == 255 ? -1 : (int)m[15]}; }
JD int64_t dec64(const Raw& r) {  // int() of [-]digits (<= 15 of them)
  int64_t v = 0;
  int k = 0;
  const bool neg = r.n > 0 && r.p[0] == '-';
  if (neg) k = 1;
  for (; k < r.n; ++k) v = 10 * v + (r.p[k] - '0');
  return neg ? -v : v;
}

struct Item {
  int msg;
  const sdx_result* rec;
};

template <class S>
JD void emit(S& o, const sdx_json_in& in, const BankView& bv, const sdx_json_rec* jt, const Item& it) {
  const sdx_result r = *it.rec;
  const sdx_json_rec j = jt[r.proto];
  o.lit("{\n    \"protocol_id\": ");
  o.bytes(bv.str + j.pid_off, j.pid_len);
  o.lit(",\n    \"payload\": \"");
  o.esc(in.heap_dev + r.payload_off, r.payload_len);
  o.lit("\",\n    \"metadata\": {\n        ");
  const uint8_t* m = in.meta_dev + 32 * (int64_t)it.msg;
  if (in.kind == SDX_KIND_MU || in.kind == SDX_KIND_MS) {  // {bit_length, rssi: R or None, clock}
    o.lit("\"bit_length\": ");
    o.u64(r.bit_length);
    o.lit(",\n        \"rssi\": ");
    const Raw R = meta_str(m);
    if (R.n < 0) {
      o.lit("null");
    } else {
      o.put('"');
      o.esc(R.p, R.n);
      o.put('"');
    }
    o.lit(",\n        \"clock\": ");
    if (in.kind == SDX_KIND_MU) {
      o.bytes(bv.str + j.s1_off, j.s1_len);  // json.dumps(float(clockabs))
    } else {  // abs(P[CP]): an integral double (the front end parses <= 15 digits)
      const double c = fabs(in.pat_val_dev[10 * (int64_t)it.msg + in.cp_slot_dev[it.msg]]);
      o.u64((uint64_t)c);
      o.put('.');
      o.put('0');
    }
  } else if (in.kind == SDX_KIND_MC) {  // {protocol_id, rssi: None, freq_afc: None}
    o.lit("\"protocol_id\": ");
    o.bytes(bv.str + j.pid_off, j.pid_len);
    o.lit(",\n        \"rssi\": null,\n        \"freq_afc\": null");
  } else {  // MN: {rssi, freq_afc, modulation, rfmode}
    o.lit("\"rssi\": ");
    const Raw R = meta_str(m), A = meta_str(m + 16);
    if (R.n <= 0) {
      o.lit("null");
    } else {  // calc_rssi: (R - 256 if R >= 128 else R) / 2 - 74
      const int64_t v = dec64(R);
      half_float(o, (v >= 128 ? v - 256 : v) - 148, false);
    }
    o.lit(",\n        \"freq_afc\": ");
    if (A.n <= 0) {
      o.lit("null");
    } else {  // round((26000000 / 16384 * A / 1000), 0) in fp64
      const double x = rint((26000000.0 / 16384.0) * (double)dec64(A) / 1000.0);
      half_float(o, 2 * (int64_t)x, x == 0.0 && signbit(x));
    }
    o.lit(",\n        \"modulation\": ");
    o.bytes(bv.str + j.s1_off, j.s1_len);
    o.lit(",\n        \"rfmode\": ");
    o.bytes(bv.str + j.s2_off, j.s2_len);
  }
  o.lit("\n    }\n}");
}

constexpr int JT = 256;

__global__ __launch_bounds__(JT) void k_json(const void* __restrict__ bank, sdx_json_in in, sdx_json_out out) {
  const BankView bv = bank_view(bank);
  const sdx_bank_hdr* h = bv.hdr;
  const uint32_t cls0 = in.kind == SDX_KIND_MU ? 0u
                        : in.kind == SDX_KIND_MS ? h->n_mu
                        : in.kind == SDX_KIND_MC ? h->n_mu + h->n_ms
                                                 : h->n_mu + h->n_ms + h->n_mc;
  const sdx_json_rec* jt = reinterpret_cast<const sdx_json_rec*>(bv.base + h->off_json) + cls0;
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * JT + threadIdx.x;
  const int nitems = in.first_only ? in.n : min((int)in.cursor_dev[0], in.rec_max);
  bool have = false;
  Item it{0, nullptr};
  if (g < nitems) {
    if (in.first_only) {
      const sdx_desc d = in.desc_dev[g];
      if (d.status == SDX_ST_OK && d.n_rec > 0) {
        have = true;
        it = Item{g, in.rec_dev + d.rec_begin};
      }
    } else {
      have = true;
      it = Item{(int)in.rec_dev[g].msg, in.rec_dev + g};
    }
  }
  uint32_t len = 0;
  if (have) {
    Count c;
    emit(c, in, bv, jt, it);
    len = c.n;
  }
  uint32_t incl = len;
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += t;
  }
  const uint32_t wtot = (uint32_t)__shfl((int)incl, WAVE - 1);
  uint32_t base = 0;
  int ovf = 0;
  if (lane == 0 && wtot) {
    base = atomicAdd(&out.cursor_dev[0], wtot);
    if ((uint64_t)base + wtot > out.json_cap) {
      ovf = 1;
      atomicOr(&out.cursor_dev[1], 1u);
    }
  }
  base = (uint32_t)__shfl((int)base, 0);
  ovf = __shfl(ovf, 0);
  if (g >= nitems) return;
  if (in.first_only == 2 && !have) return;   // sparse: only the lines with a text (kinds share the outputs)
  const uint32_t off = base + incl - len;
  out.off_dev[g] = off;
  out.len_dev[g] = ovf ? 0u : len;
  if (!have || ovf) return;
  J8 w(out.json_dev + off);
  emit(w, in, bv, jt, it);
  w.finish();
}

}  // namespace sdxj

extern "C" int sdx_serialize_json(const sdx_bank* bank, const sdx_json_in* in, const sdx_json_out* out,
                                  void* hip_stream) {
  if (!bank || !in || !out) return sdx::set_error(SDX_EINVAL, "sdx_serialize_json: null argument");
  if (in->kind < SDX_KIND_MU || in->kind > SDX_KIND_MN)
    return sdx::set_error(SDX_EINVAL, "sdx_serialize_json: bad kind");
  if (!in->desc_dev || !in->rec_dev || !in->cursor_dev || !in->heap_dev || !in->meta_dev || !out->json_dev ||
      !out->off_dev || !out->len_dev || !out->cursor_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_serialize_json: null buffer");
  if (in->kind == SDX_KIND_MS && (!in->pat_val_dev || !in->cp_slot_dev))
    return sdx::set_error(SDX_EINVAL, "sdx_serialize_json: MS needs pat_val/cp_slot");
  const int items = in->first_only ? in->n : in->rec_max;
  if (items <= 0) return SDX_OK;
  hipLaunchKernelGGL(sdxj::k_json, dim3((items + sdxj::JT - 1) / sdxj::JT), dim3(sdxj::JT), 0,
                     (hipStream_t)hip_stream, sdx::bank_dev_ptr(bank), *in, *out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_serialize_json: ") + hipGetErrorString(e));
  return SDX_OK;
}
