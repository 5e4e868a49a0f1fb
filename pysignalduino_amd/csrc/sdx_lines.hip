// sdx_lines.hip -- the wire-line front end, hand-written HIP for gfx950.
//
// Raw firmware lines -> demodulator batches, one lane per line, entirely on the device.  Per line
// this restates what the reference does before demodulation:
//   transport.py:123            bytes.decode("latin-1").strip()  (bytes here = the latin-1 string)
//   parser/__init__.py:37-49    SignalParser.parse_line: extract_payload, route by payload[:2].upper()
//   parser/base.py:188-206      extract_payload: strip, ^\x02(M[sSuUcCNOo];.*;)\x03$
//   parser/base.py:13-186       decompress_payload (Mred=1 lines)
//   parser/mu.py:48-68          the MU validity regex, _parse_to_dict, "D" required
//   parser/ms.py:35-41          _parse_to_dict, "D" required
//   parser/mc.py:37-155         MC header validation, required D/C/L, hex D, int(R)/int(F)
//   sd_protocols/message_*.py   the P#/CP/SP/R/data string gates the demodulators apply
// The outputs of line i are message i of an sdx_pulse_batch / sdx_mc_batch in slot layout
// (len_dev), so the demodulation kernels read them in place.  Anything whose exact Python meaning
// this file does not model (bytes >= 0x80 after decompression, multi-digit pattern ids, non-integer
// pattern values, MN lines) is reported SDX_LS_UNSUPPORTED instead of being approximated.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/sdx.h"

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
}

namespace sdxl {

#define LD __device__ __forceinline__

struct Str {
  const uint8_t* p;
  int n;
};

// Python character classes on a latin-1 character (tables checked in tests/test_lines.py)
LD bool py_space(uint8_t c) { return (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x20) || c == 0x85 || c == 0xa0; }
LD bool digit(uint8_t c) { return c >= '0' && c <= '9'; }
LD bool hexc(uint8_t c) { return digit(c) || ((c | 32) >= 'a' && (c | 32) <= 'f'); }
LD bool py_alpha(uint8_t c) {
  if ((c | 32) >= 'a' && (c | 32) <= 'z') return true;
  return c == 0xaa || c == 0xb5 || c == 0xba || (c >= 0xc0 && c <= 0xd6) || (c >= 0xd8 && c <= 0xf6) || c >= 0xf8;
}
LD bool py_alnum_ascii(uint8_t c) { return c < 128 && (digit(c) || ((c | 32) >= 'a' && (c | 32) <= 'z')); }
LD uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }
LD int hexv(uint8_t c) { return digit(c) ? c - '0' : ((c | 32) - 'a' + 10); }

struct Writer {
  uint8_t* d;
  int n, cap;
  bool ovf;
  LD void put(uint8_t c) {
    if (n < cap) d[n] = c;
    else ovf = true;
    ++n;
  }
  LD void put_uint(uint32_t v) {
    char t[10];
    int k = 0;
    do {
      t[k++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    while (k) put((uint8_t)t[--k]);
  }
};

// next non-empty ';'-separated part at or after pos: [s, e); returns false at the end
LD bool next_part(const Str& P, int& pos, int& s, int& e) {
  while (pos <= P.n) {
    s = pos;
    e = s;
    while (e < P.n && P.p[e] != ';') ++e;
    pos = e + 1;
    if (e > s) return true;
  }
  return false;
}

// base.py:76-99: does this part end the merged D= payload?
LD bool d_field(const Str& P, int s, int e) {
  const uint8_t m0 = P.p[s];
  const int m1n = e - s - 1;
  if (!py_alpha(m0)) return false;
  if (m0 == 'D' || m0 == 'd') return true;
  if (m0 > 127) return true;
  if (m0 == 'M') return true;
  if ((m0 == 'C' || m0 == 'S') && m1n == 1) return true;
  if (m0 == 'o' || m0 == 'm') return true;
  if (m1n >= 1 && m1n <= 2 && hexc(P.p[s + 1]) && (m1n == 1 || hexc(P.p[s + 2]))) return true;
  for (int i = s; i < e; ++i)
    if (P.p[i] == '=') return true;  // alnum (ASCII letter here) and '=' in the part
  return false;
}

// decompress_payload (base.py:13-186) into w; returns false when an upper() of a non-ASCII
// character would be needed (UNSUPPORTED)
LD bool decompress(const Str& P, Writer& w) {
  int pos = 0, s, e;
  bool first = true;
  while (next_part(P, pos, s, e)) {
    const uint8_t m0 = P.p[s];
    const int m1s = s + 1, m1n = e - s - 1;
    const int mark = w.n;
    if (!first) w.put(';');
    bool emitted = true;
    if (m0 == 'D' || m0 == 'd') {  // :59-140, with the merge of ';'-split binary data
      w.put('D');
      w.put('=');
      const int d0 = w.n;
      auto emit_byte = [&](uint8_t c) {
        w.put_uint((c >> 4) & 0xF);
        w.put((uint8_t)('0' + (c & 0x7)));
      };
      for (int i = m1s; i < e; ++i) emit_byte(P.p[i]);
      int j = pos, s2, e2;
      while (true) {
        const int before = j;
        if (!next_part(P, j, s2, e2)) {
          pos = j;
          break;
        }
        if (d_field(P, s2, e2)) {
          pos = before;  // the loop resumes at this part
          break;
        }
        emit_byte(';');  // cur += ';' + next_part (empty parts in between are dropped)
        for (int i = s2; i < e2; ++i) emit_byte(P.p[i]);
        pos = j;
      }
      if (m0 == 'd' && w.n > d0) w.n -= 1;  // :130-131
      if (w.n > d0 && w.n <= w.cap && w.d[d0] == '8') {  // :134-135
        for (int i = d0; i + 1 < w.n && i + 1 < w.cap; ++i) w.d[i] = w.d[i + 1];
        w.n -= 1;
      }
    } else if (m0 == 'M') {  // :144-146
      w.put('M');
      for (int i = m1s; i < e; ++i) {
        if (P.p[i] >= 128) return false;
        w.put(up(P.p[i]));
      }
    } else if (m0 > 127) {  // :149-165
      w.put('P');
      w.put((uint8_t)('0' + (m0 & 7)));
      w.put('=');
      if (m1n == 2) {
        uint32_t ml = P.p[m1s] & 127, mh = P.p[m1s + 1] & 127;
        if (m0 & 32) w.put('-');
        if (m0 & 16) ml += 128;
        w.put_uint(mh * 256 + ml);
      }
    } else if ((m0 == 'C' || m0 == 'S') && m1n == 1) {  // :168-169
      w.put(m0);
      w.put('P');
      w.put('=');
      w.put(P.p[m1s]);
    } else if (m0 == 'o' || m0 == 'm') {  // :172-173
      for (int i = s; i < e; ++i) w.put(P.p[i]);
    } else if (m1n >= 1 && m1n <= 2 && hexc(P.p[m1s]) && (m1n == 1 || hexc(P.p[m1s + 1]))) {  // :176-177
      w.put(m0);
      w.put('=');
      w.put_uint(m1n == 1 ? hexv(P.p[m1s]) : 16 * hexv(P.p[m1s]) + hexv(P.p[m1s + 1]));
    } else if (py_alnum_ascii(m0)) {  // :180-181
      w.put(m0);
      if (m1n) w.put('=');
      for (int i = m1s; i < e; ++i) w.put(P.p[i]);
    } else {
      emitted = false;
    }
    if (emitted) first = false;
    else w.n = mark;  // no part, no separator
  }
  w.put(';');  // :184
  return true;
}

LD bool lit(const Str& P, int pos, const char* s) {
  for (int i = 0; s[i]; ++i)
    if (pos + i >= P.n || P.p[pos + i] != (uint8_t)s[i]) return false;
  return true;
}
LD int digits_at(const Str& P, int pos) {
  int k = 0;
  while (pos + k < P.n && digit(P.p[pos + k])) ++k;
  return k;
}

// parser/mu.py:48 ^(?=.*D=\d+)(?:MU;(?:P[0-7]=-?[0-9]{1,5};){2,8}((?:D=\d{2,};)|(?:CP=\d;)|(?:R=\d+;)|
// (?:O;)|(?:e;)|(?:p;)|(?:w=\d;))*)$  -- no item can start like another, so one left-to-right scan
// decides it (and with a D item present the lookahead holds)
LD bool mu_valid(const Str& P) {
  int n = P.n;
  if (n > 0 && P.p[n - 1] == '\n') --n;  // '$' also matches before a final newline
  Str Q{P.p, n};
  if (!lit(Q, 0, "MU;")) return false;
  int pos = 3, np = 0;
  while (pos < n && Q.p[pos] == 'P') {
    if (np == 8) return false;  // a ninth P item cannot match anything
    if (pos + 2 >= n || Q.p[pos + 1] < '0' || Q.p[pos + 1] > '7' || Q.p[pos + 2] != '=') return false;
    int q = pos + 3;
    if (q < n && Q.p[q] == '-') ++q;
    const int k = digits_at(Q, q);
    if (k < 1 || k > 5 || q + k >= n || Q.p[q + k] != ';') return false;
    pos = q + k + 1;
    ++np;
  }
  if (np < 2) return false;
  bool hasd = false;
  while (pos < n) {
    const uint8_t c = Q.p[pos];
    if (c == 'D' && lit(Q, pos, "D=")) {
      const int k = digits_at(Q, pos + 2);
      if (k < 2 || pos + 2 + k >= n || Q.p[pos + 2 + k] != ';') return false;
      pos += 3 + k;
      hasd = true;
    } else if (c == 'C' && lit(Q, pos, "CP=")) {
      if (pos + 4 >= n || !digit(Q.p[pos + 3]) || Q.p[pos + 4] != ';') return false;
      pos += 5;
    } else if (c == 'R' && lit(Q, pos, "R=")) {
      const int k = digits_at(Q, pos + 2);
      if (k < 1 || pos + 2 + k >= n || Q.p[pos + 2 + k] != ';') return false;
      pos += 3 + k;
    } else if ((c == 'O' || c == 'e' || c == 'p') && pos + 1 < n && Q.p[pos + 1] == ';') {
      pos += 2;
    } else if (c == 'w' && lit(Q, pos, "w=")) {
      if (pos + 3 >= n || !digit(Q.p[pos + 2]) || Q.p[pos + 3] != ';') return false;
      pos += 4;
    } else {
      return false;
    }
  }
  return hasd;
}

// int value of [-+]?[0-9]{1,15} (exact as a double); 0 = empty, 1 = ok, 2 = something else
LD int parse_int15(const Str& P, int s, int e, long long* v) {
  if (s == e) return 0;
  int i = s;
  bool neg = false;
  if (P.p[i] == '-' || P.p[i] == '+') {
    neg = P.p[i] == '-';
    ++i;
  }
  if (i == e || e - i > 15) return 2;
  long long x = 0;
  for (; i < e; ++i) {
    if (!digit(P.p[i])) return 2;
    x = 10 * x + (P.p[i] - '0');
  }
  *v = neg ? -x : x;
  return 1;
}
// int() of [-+]?[0-9]+ (any length): 0 = empty, 1 = ok, 2 = not decimal, 3 = ok but |v| >= 2^31
LD int parse_dec(const Str& P, int s, int e, long long* v) {
  if (s == e) return 0;
  int i = s;
  bool neg = false;
  if (P.p[i] == '-' || P.p[i] == '+') {
    neg = P.p[i] == '-';
    ++i;
  }
  if (i == e) return 2;
  long long x = 0;
  bool big = false;
  for (; i < e; ++i) {
    if (!digit(P.p[i])) return 2;
    x = 10 * x + (P.p[i] - '0');
    if (x >= (1ll << 31)) {
      big = true;
      x = 1ll << 31;
    }
  }
  *v = neg ? -x : x;
  return big && !(neg && x == (1ll << 31)) ? 3 : 1;
}
LD bool all_digits(const Str& P, int s, int e) {
  if (s >= e) return false;
  for (int i = s; i < e; ++i)
    if (!digit(P.p[i])) return false;
  return true;
}
LD bool keq(const Str& P, int s, int e, const char* k) {
  int i = 0;
  for (; k[i]; ++i)
    if (s + i >= e || P.p[s + i] != (uint8_t)k[i]) return false;
  return s + i == e;
}

struct Field {
  int s, e;  // value range, s < 0: absent
};


// ---- the parse kernel -------------------------------------------------------------------------
// One lane per line.  A wave first stages the byte span of its (next) lines into its own LDS region
// with coalesced 16-byte loads, then every lane scans its line in LDS; compressed payloads are
// decompressed into a per-wave LDS area (prefix-sum allocated), and at the end of a round the
// wave copies each line's D characters (or whole decompressed payload) to the slot with
// byte-consecutive stores.  A line longer than the stage buffer, or a payload whose decompression
// does not fit the LDS area, takes the same code on global memory (exact, slower).
constexpr int PW = 2;         // waves per workgroup
constexpr int STAGE = 8192;   // staged line bytes per wave and round
constexpr int DECB = 4096;    // decompressed payload bytes per wave and round

struct alignas(16) ParseLds {
  uint8_t stage[STAGE + 32];
  uint8_t dec[DECB];
  uint32_t pv[10 * 64];  // fast P-key table [id][lane]: last value start | end << 16
};

struct LineRes {
  uint8_t kind = SDX_LINE_NONE, status = SDX_LS_NOFRAME;
  int dS = 0, dE = 0;  // D (MU/MS) or hex (MC) characters in the payload
  Field fR{-1, -1}, fF{-1, -1};
};

LD void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

LD int64_t shfl64(int64_t v, int src) {
  const int lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), src);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// extract_payload (base.py:188-206): payload = L[pa, pa + pn); also whether decompress_payload
// runs on it (MS/MU/MO/MN with a byte >= 0x80 after the header).  One pass over the bytes.
LD bool frame_line(const uint8_t* L, int len, int& pa, int& pn, bool& comp) {
  int a = 0, b = len;
  while (a < b && py_space(L[a])) ++a;
  while (b > a && py_space(L[b - 1])) --b;
  if (b - a < 6 || L[a] != 0x02 || L[b - 1] != 0x03 || L[a + 1] != 'M' || L[a + 3] != ';' || L[b - 2] != ';')
    return false;
  const uint8_t t = L[a + 2];
  if (!(t == 's' || t == 'S' || t == 'u' || t == 'U' || t == 'c' || t == 'C' || t == 'N' || t == 'O' || t == 'o'))
    return false;
  uint8_t any = 0;
  for (int k = a + 4; k < b - 2; ++k) {  // '.' does not match a newline
    const uint8_t c = L[k];
    if (c == '\n') return false;
    any |= c;
  }
  const uint8_t t1 = up(t);
  comp = (any & 0x80) && (t1 == 'S' || t1 == 'U' || t1 == 'O' || t1 == 'N');
  pa = a + 1;
  pn = b - a - 2;
  return true;
}

LD bool same_key(const Str& P, int s1, int e1, int s2, int e2) {
  if (e1 - s1 != e2 - s2) return false;
  for (int k = 0; k < e1 - s1; ++k)
    if (P.p[s1 + k] != P.p[s2 + k]) return false;
  return true;
}

// routing + the per-type parser rules on a (decompressed) payload; writes the pattern / MS / MC
// fields of line i, returns kind/status and the D/R/F ranges.  pvt = this lane's column of the
// fast P-key table (stride 64 words).
LD void parse_payload(const Str& P, LineRes& r, const sdx_lines_out& out, int i, uint32_t* pvt) {
  // ---- routing: payload[:2].upper()
  const uint8_t c0 = P.n > 0 ? up(P.p[0]) : 0, c1 = P.n > 1 ? up(P.p[1]) : 0;
  if (c0 != 'M' || !(c1 == 'S' || c1 == 'U' || c1 == 'C' || c1 == 'N')) {
    r.status = SDX_LS_NOPARSER;
    return;
  }
  r.kind = c1 == 'U' ? SDX_LINE_MU : c1 == 'S' ? SDX_LINE_MS : c1 == 'C' ? SDX_LINE_MC : SDX_LINE_MN;
  if (r.kind == SDX_LINE_MN) {  // the MN (FSK) path is not part of this build
    r.status = SDX_LS_UNSUPPORTED;
    return;
  }
  {
    uint8_t any = 0;
    for (int k = 0; k < P.n; ++k) any |= P.p[k];
    if (any & 0x80) {  // str methods on non-ASCII characters are not modelled
      r.status = SDX_LS_UNSUPPORTED;
      return;
    }
  }
  if (r.kind == SDX_LINE_MU && !mu_valid(P)) {
    r.status = SDX_LS_INVALID;
    return;
  }
  Field fD{-1, -1}, fCP{-1, -1}, fSP{-1, -1}, fC{-1, -1}, fL{-1, -1};
  Field& fR = r.fR;
  Field& fF = r.fF;
  if (r.kind == SDX_LINE_MC) {
    // ---- MCParser._parse_to_dict + key set + required fields (mc.py:37-56,95-139)
    int pos = 0, s, e;
    uint32_t seen = 0;  // LL LH SL SH D C L R F M MC Mc
    while (next_part(P, pos, s, e)) {
      int eq = -1;
      for (int k = s; k < e; ++k)
        if (P.p[k] == '=') {
          eq = k;
          break;
        }
      int bit = -1;
      if (eq >= 0) {
        const int kl = eq - s;
        bool keyok = kl >= 1 && kl <= 2;
        for (int k = s; k < eq && keyok; ++k) keyok = P.p[k] >= 'A' && P.p[k] <= 'Z';
        int v = eq + 1;
        if (v < e && (P.p[v] == '-' || P.p[v] == '+')) ++v;
        bool valok = v < e;
        for (int k = v; k < e && valok; ++k) valok = hexc(P.p[k]);
        if (!keyok || !valok) {
          r.status = SDX_LS_INVALID;
          return;
        }
        static const char* const KEYS[11] = {"LL", "LH", "SL", "SH", "D", "C", "L", "R", "F", "M", "MC"};
        for (int q = 0; q < 11 && bit < 0; ++q)
          if (keq(P, s, eq, KEYS[q])) bit = q;
        if (bit < 0) {  // a well-formed key outside the MC header set
          r.status = SDX_LS_INVALID;
          return;
        }
        const Field f{eq + 1, e};
        if (bit == 4) fD = f;
        if (bit == 5) fC = f;
        if (bit == 6) fL = f;
        if (bit == 7) fR = f;
        if (bit == 8) fF = f;
      } else {
        if (keq(P, s, e, "MC")) bit = 10;
        else if (keq(P, s, e, "Mc")) bit = 11;
        else {  // not MC/Mc: invalid after the first part, and outside the key set as the first
          r.status = SDX_LS_INVALID;
          return;
        }
      }
      if (seen & (1u << bit)) {  // duplicate key
        r.status = SDX_LS_INVALID;
        return;
      }
      seen |= 1u << bit;
    }
    if (fD.s < 0 || fC.s < 0 || fL.s < 0) {
      r.status = SDX_LS_INVALID;
      return;
    }
    for (int k = fD.s; k < fD.e; ++k)  // re.fullmatch(r"[0-9a-fA-F]+", raw_hex)
      if (!hexc(P.p[k])) {
        r.status = SDX_LS_INVALID;
        return;
      }
    long long v;
    const int rr = fR.s >= 0 ? parse_dec(P, fR.s, fR.e, &v) : 1, rf = fF.s >= 0 ? parse_dec(P, fF.s, fF.e, &v) : 1;
    if ((rr != 1 && rr != 3) || (rf != 1 && rf != 3)) {  // int(R) / int(F) raise -> ignored (mc.py:141-155)
      r.status = SDX_LS_INVALID;
      return;
    }
    long long cv = 0, lv = 0;
    const int rc = parse_dec(P, fC.s, fC.e, &cv), rl = parse_dec(P, fL.s, fL.e, &lv);
    if (rc == 2 || rl == 2) {  // int(C) / int(L) raise inside demodulate_mc -> caught, nothing decoded
      r.status = SDX_LS_RAISES;
      return;
    }
    if (rc != 1 || rl != 1 || fD.e - fD.s > SDX_MC_HEX_MAX) {  // outside the int32 / frame-length contract
      r.status = SDX_LS_UNSUPPORTED;
      return;
    }
    out.clock_dev[i] = (int32_t)cv;
    out.mcbitnum_dev[i] = (int32_t)lv;
    out.mcflags_dev[i] = 0;  // msg_data.get("M", "MC") is never "Mc" (mc.py:60); no version
  } else {
    // ---- _parse_to_dict (mu.py:82-94, ms.py:65-78): last value wins, first position counts.
    // P-keys "P<d>" (one digit) go to the lane's LDS table; any longer P-key ("P05", "P10")
    // switches to the general (nested-scan) form below.
    int pos = 0, s, e;
    uint32_t seen = 0;
    uint64_t order = 0;
    int nord = 0;
    bool slow = P.n > 0xFFFF;
    while (next_part(P, pos, s, e)) {
      int eq = -1;
      for (int k = s; k < e; ++k)
        if (P.p[k] == '=') {
          eq = k;
          break;
        }
      const int ke = eq >= 0 ? eq : e;
      const Field f{eq >= 0 ? eq + 1 : e, e};
      if (keq(P, s, ke, "D")) fD = f;
      else if (keq(P, s, ke, "CP")) fCP = f;
      else if (keq(P, s, ke, "SP")) fSP = f;
      else if (keq(P, s, ke, "R")) fR = f;
      else if (keq(P, s, ke, "F")) fF = f;
      else if (P.p[s] == 'P' && ke - s >= 2 && all_digits(P, s + 1, ke)) {
        if (ke - s == 2 && !slow) {
          const int d = P.p[s + 1] - '0';
          if (!((seen >> d) & 1)) {
            seen |= 1u << d;
            order |= (uint64_t)d << (4 * nord);
            ++nord;
          }
          pvt[64 * d] = (uint32_t)f.s | ((uint32_t)f.e << 16);
        } else {
          slow = true;
        }
      }
    }
    if (fD.s < 0) {  // "D" not in msg_data
      r.status = SDX_LS_NODATA;
      return;
    }
    // message_synced.py:21-47 string gates (packing.PulsePacker.add); patterns are converted only
    // where the reference converts them (MS past the gates, MU with non-empty data)
    bool ms_ok = r.kind == SDX_LINE_MS && all_digits(P, fD.s, fD.e) && fCP.s >= 0 && all_digits(P, fCP.s, fCP.e) &&
                 fSP.s >= 0 && all_digits(P, fSP.s, fSP.e) && (fR.s < 0 || all_digits(P, fR.s, fR.e));
    const bool want_pat = r.kind == SDX_LINE_MS ? ms_ok : fD.e > fD.s;
    // _patterns (message_unsynced.py:28-35): id = str(int(k[1:])), value = float(v), ValueError
    // skipped; slot = first successful assignment of the id, value = the last one
    int nslot = 0;
    uint64_t sidp = 0;  // slot z -> id in nibble z
    double* pval = out.pat_val_dev + 10 * (int64_t)i;
    uint8_t* pid = out.pat_id_dev + 10 * (int64_t)i;
    auto assign = [&](int id, double v) {
      int z = 0;
      while (z < nslot && (int)((sidp >> (4 * z)) & 15) != id) ++z;
      if (z == nslot) {
        sidp |= (uint64_t)id << (4 * z);
        pid[z] = (uint8_t)('0' + id);
        ++nslot;
      }
      pval[z] = v;
    };
    if (want_pat && !slow) {
      for (int q = 0; q < nord; ++q) {
        const int d = (int)((order >> (4 * q)) & 15);
        const uint32_t w = pvt[64 * d];
        long long v;
        const int rv = parse_int15(P, (int)(w & 0xFFFF), (int)(w >> 16), &v);
        if (rv == 0) continue;  // float('') -> ValueError -> skipped
        if (rv == 2) {          // other float() syntax: not modelled
          r.status = SDX_LS_UNSUPPORTED;
          return;
        }
        assign(d, (double)v);
      }
    } else if (want_pat) {
      pos = 0;
      while (next_part(P, pos, s, e)) {
        int eq = -1;
        for (int k = s; k < e; ++k)
          if (P.p[k] == '=') {
            eq = k;
            break;
          }
        const int ke = eq >= 0 ? eq : e;
        if (!(P.p[s] == 'P' && ke - s >= 2 && all_digits(P, s + 1, ke))) continue;
        bool dup = false;  // msg_data holds each key string once, at its first position
        int p2 = 0, s2, e2;
        while (!dup && next_part(P, p2, s2, e2) && s2 < s) {
          int k2 = s2;
          while (k2 < e2 && P.p[k2] != '=') ++k2;
          dup = same_key(P, s, ke, s2, k2);
        }
        if (dup) continue;
        int vs = eq >= 0 ? eq + 1 : e, ve = e;  // ... with the value of its last occurrence
        int p3 = pos, s3, e3;
        while (next_part(P, p3, s3, e3)) {
          int k3 = s3;
          while (k3 < e3 && P.p[k3] != '=') ++k3;
          if (same_key(P, s, ke, s3, k3)) {
            vs = k3 < e3 ? k3 + 1 : e3;
            ve = e3;
          }
        }
        long long idv = 0;
        for (int k = s + 1; k < ke; ++k)
          if (idv < 1000) idv = 10 * idv + (P.p[k] - '0');
        long long v;
        const int rv = parse_int15(P, vs, ve, &v);
        if (rv == 0) continue;
        if (rv == 2 || idv >= 10) {  // other float() syntax / a multi-character pattern id
          r.status = SDX_LS_UNSUPPORTED;
          return;
        }
        assign((int)idv, (double)v);
      }
    }
    if (fD.e - fD.s > SDX_LONG_MAX) {  // longer than the long demodulation variant takes
      r.status = SDX_LS_UNSUPPORTED;
      return;
    }
    out.npat_dev[i] = (uint8_t)nslot;
    if (r.kind == SDX_LINE_MS) {
      int8_t slotv = -1;
      if (ms_ok) {  // str(int(CP)) in the pattern ids, else no demodulation
        long long cp = 0;
        for (int k = fCP.s; k < fCP.e; ++k)
          if (cp < 1000) cp = 10 * cp + (P.p[k] - '0');
        for (int z = 0; z < nslot; ++z)
          if (cp < 10 && (int)((sidp >> (4 * z)) & 15) == cp) slotv = (int8_t)z;
        ms_ok = slotv >= 0;
      }
      out.cp_slot_dev[i] = slotv;
      out.ms_ok_dev[i] = ms_ok ? 1 : 0;
    }
  }
  if ((fR.s >= 0 && fR.e - fR.s > 15) || (fF.s >= 0 && fF.e - fF.s > 15)) {  // meta_dev holds 15 bytes
    r.status = SDX_LS_UNSUPPORTED;
    return;
  }
  r.dS = fD.s;
  r.dE = fD.e;
  r.status = SDX_LS_OK;
}

// 16 bytes of meta_dev: value characters, length at byte 15 (255 = absent)
LD uint4 meta16(const Str& P, Field f) {
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  if (f.s < 0) {
    w3 = 255u << 24;
  } else {
    const int n = f.e - f.s;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const uint32_t c = k < n ? (uint32_t)P.p[f.s + k] << (8 * (k & 3)) : 0u;
      if (k < 4) w0 |= c;
      else if (k < 8) w1 |= c;
      else if (k < 12) w2 |= c;
      else w3 |= c;
    }
    w3 |= (uint32_t)n << 24;
  }
  return make_uint4(w0, w1, w2, w3);
}

LD void finish_fields(const Str& P, const LineRes& r, const sdx_lines_out& out, int i) {
  uint4* m = reinterpret_cast<uint4*>(out.meta_dev + 32 * (int64_t)i);
  m[0] = meta16(P, r.fR);
  m[1] = meta16(P, r.fF);
  out.dlen_dev[i] = r.dE - r.dS;
}

// a line on global memory only (longer than the stage buffer): same rules, lane-serial copy
LD void line_global(const sdx_lines& in, const sdx_lines_out& out, int i, int64_t lo, int64_t hi, uint32_t* pvt) {
  const uint8_t* L = in.bytes_dev + lo;
  LineRes r;
  int pa = 0, pn = 0;
  bool comp = false;
  int plen = -1;
  int64_t doff = 3 * lo;
  if (frame_line(L, (int)(hi - lo), pa, pn, comp)) {
    Str P{L + pa, pn};
    uint8_t* slot = out.slot_dev + 3 * lo;
    bool ok = true;
    if (comp) {
      Writer w{slot, 0, (int)(3 * (hi - lo)), false};
      ok = decompress(P, w) && !w.ovf;
      P = Str{slot, w.n};
      plen = w.n;
    }
    if (!ok) {
      r.status = SDX_LS_UNSUPPORTED;
    } else {
      parse_payload(P, r, out, i, pvt);
      if (r.status == SDX_LS_OK) {
        if (comp) {
          doff = 3 * lo + r.dS;
        } else {
          for (int k = 0; k < r.dE - r.dS; ++k) slot[k] = P.p[r.dS + k];
        }
        finish_fields(P, r, out, i);
      }
    }
  }
  out.doff_dev[i] = doff;
  out.plen_dev[i] = plen;
  out.kind_dev[i] = r.kind;
  out.status_dev[i] = r.status;
}

__global__ __launch_bounds__(64 * PW) void k_parse_lines(sdx_lines in, sdx_lines_out out) {
  __shared__ ParseLds sm[PW];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  ParseLds& S = sm[wave];
  const int first = (blockIdx.x * PW + wave) * 64;
  if (first >= in.n) return;  // wave-uniform
  const int nv = min(64, in.n - first);
  const int i = first + lane;
  const bool valid = lane < nv;
  const int64_t total = in.offsets_dev[in.n];
  int64_t lo = 0, hi = 0;
  if (valid) {
    lo = in.offsets_dev[i];
    hi = in.offsets_dev[i + 1];
  }
  uint32_t* pvt = S.pv + lane;
  uint8_t* const sbase = reinterpret_cast<uint8_t*>(&S);
  int next = 0;
  while (next < nv) {
    const int64_t base = shfl64(lo, next);
    const bool fits = valid && lane >= next && hi - base <= STAGE;
    const int k = next + __popcll(__ballot(fits));  // hi is monotone: the fitting lanes are next..k-1
    if (k == next) {  // line `next` alone exceeds the stage buffer
      if (lane == next) line_global(in, out, i, lo, hi, pvt);
      ++next;
      continue;
    }
    // ---- stage bytes [base, end) with 16-byte loads: LDS byte j <-> global byte (ga + j)
    const int64_t end = shfl64(hi, k - 1);
    const uint8_t* gb = in.bytes_dev + base;
    const int sh = (int)((uintptr_t)gb & 15);
    const uint8_t* ga = gb - sh;
    const int nch = (int)((end - base + sh + 15) >> 4);
    const uint8_t* glo = in.bytes_dev;
    const uint8_t* ghi = in.bytes_dev + total;
    for (int c = lane; c < nch; c += 64) {
      const uint8_t* src = ga + 16 * c;
      if (src >= glo && src + 16 <= ghi) {
        *reinterpret_cast<uint4*>(S.stage + 16 * c) = *reinterpret_cast<const uint4*>(src);
      } else {
        for (int q = 0; q < 16; ++q) S.stage[16 * c + q] = (src + q >= glo && src + q < ghi) ? src[q] : 0;
      }
    }
    wave_sync();
    const bool mine = lane >= next && lane < k;
    LineRes r;
    int pa = 0, pn = 0;
    bool comp = false, framed = false;
    const uint8_t* L = S.stage + sh + (lo - base);
    if (mine) framed = frame_line(L, (int)(hi - lo), pa, pn, comp);
    // decompression targets: prefix-sum allocation in the wave's LDS area, else the global slot
    const int ub = (mine && framed && comp) ? 3 * pn + 16 : 0;
    int incl = ub;
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    const int doff_l = incl - ub;
    const bool dec_lds = incl <= DECB;
    int plen = -1;
    int64_t doff = 3 * lo;
    uint32_t cp_src = 0;
    int cp_len = 0;
    if (mine && framed) {
      const Str Ps{L + pa, pn};
      if (comp && !dec_lds) {  // the LDS area is full: decompress into the slot and parse there
        uint8_t* slot = out.slot_dev + 3 * lo;
        Writer w{slot, 0, (int)(3 * (hi - lo)), false};
        if (!decompress(Ps, w) || w.ovf) {
          r.status = SDX_LS_UNSUPPORTED;
        } else {
          const Str P{slot, w.n};
          plen = w.n;
          parse_payload(P, r, out, i, pvt);
          if (r.status == SDX_LS_OK) {
            doff = 3 * lo + r.dS;
            finish_fields(P, r, out, i);
          }
        }
      } else {
        bool ok = true;
        Str P = Ps;
        if (comp) {
          Writer w{S.dec + doff_l, 0, ub, false};
          ok = decompress(Ps, w) && !w.ovf;
          P = Str{S.dec + doff_l, w.n};
          plen = w.n;
        }
        if (!ok) {
          r.status = SDX_LS_UNSUPPORTED;
        } else {
          parse_payload(P, r, out, i, pvt);
          if (r.status == SDX_LS_OK) {
            finish_fields(P, r, out, i);
            if (comp) {  // the whole payload goes to the slot (RawFrame.line), D inside it
              doff = 3 * lo + r.dS;
              cp_src = (uint32_t)(P.p - sbase);
              cp_len = P.n;
            } else {
              cp_src = (uint32_t)(P.p + r.dS - sbase);
              cp_len = r.dE - r.dS;
            }
          }
        }
      }
    }
    if (mine) {
      out.doff_dev[i] = doff;
      out.plen_dev[i] = plen;
      out.kind_dev[i] = r.kind;
      out.status_dev[i] = r.status;
    }
    wave_sync();
    // ---- copy-out: one line at a time, 64 consecutive bytes per store instruction
    uint64_t cm = __ballot(cp_len > 0);
    while (cm) {
      const int j = __builtin_ctzll(cm);
      cm &= cm - 1;
      const uint8_t* src = sbase + __shfl((int)cp_src, j);
      uint8_t* dst = out.slot_dev + 3 * shfl64(lo, j);
      const int len = __shfl(cp_len, j);
      for (int q = lane; q < len; q += 64) dst[q] = src[q];
    }
    wave_sync();
    next = k;
  }
}

// ---- selection lists (sdx_select_lines): class of a parsed line, -1 = not demodulated
LD int sel_class(const sdx_lines_out& o, int i) {
  if (o.status_dev[i] != SDX_LS_OK) return -1;
  const uint8_t k = o.kind_dev[i];
  const int32_t n = o.dlen_dev[i];
  if (k == SDX_LINE_MU) return n <= SDX_SHORT_MAX ? SDX_SEL_MU_SHORT : SDX_SEL_MU_LONG;
  if (k == SDX_LINE_MS) {
    if (!o.ms_ok_dev[i]) return -1;
    return n <= SDX_SHORT_MAX ? SDX_SEL_MS_SHORT : SDX_SEL_MS_LONG;
  }
  if (k == SDX_LINE_MC) return SDX_SEL_MC;
  return -1;
}

constexpr int SEL_THREADS = 256;
static_assert(SDX_SEL_CHUNK % SEL_THREADS == 0, "chunk = whole rounds of the workgroup");

// per-chunk class counts -> scratch[chunk * 8 + class]
__global__ __launch_bounds__(SEL_THREADS) void k_sel_count(sdx_lines_out o, int n, int32_t* scratch) {
  __shared__ int32_t c[SDX_SEL_NCLASS];
  if (threadIdx.x < SDX_SEL_NCLASS) c[threadIdx.x] = 0;
  __syncthreads();
  int mine[SDX_SEL_NCLASS] = {0, 0, 0, 0, 0};
  const int base = blockIdx.x * SDX_SEL_CHUNK;
  for (int r = 0; r < SDX_SEL_CHUNK; r += SEL_THREADS) {
    const int i = base + r + threadIdx.x;
    const int k = i < n ? sel_class(o, i) : -1;
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) mine[q] += k == q;
  }
#pragma unroll
  for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
    int v = mine[q];
    for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&c[q], v);
  }
  __syncthreads();
  if (threadIdx.x < 8) scratch[blockIdx.x * 8 + threadIdx.x] = threadIdx.x < SDX_SEL_NCLASS ? c[threadIdx.x] : 0;
}

// ordered write: chunk b's entries of class k go to start_k + (class-k lines of chunks < b) + rank in chunk
__global__ __launch_bounds__(SEL_THREADS) void k_sel_write(sdx_lines_out o, int n, int nchunk,
                                                           const int32_t* scratch, int32_t* sel, int32_t* counts) {
  __shared__ int32_t tot[SDX_SEL_NCLASS], pre[SDX_SEL_NCLASS], wcnt[SEL_THREADS / 64][SDX_SEL_NCLASS];
  if (threadIdx.x < SDX_SEL_NCLASS) tot[threadIdx.x] = pre[threadIdx.x] = 0;
  __syncthreads();
  {
    int t[SDX_SEL_NCLASS] = {0, 0, 0, 0, 0}, p[SDX_SEL_NCLASS] = {0, 0, 0, 0, 0};
    for (int b = threadIdx.x; b < nchunk; b += SEL_THREADS)
#pragma unroll
      for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
        const int v = scratch[b * 8 + q];
        t[q] += v;
        if (b < (int)blockIdx.x) p[q] += v;
      }
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
      int a = t[q], c = p[q];
      for (int d = 32; d; d >>= 1) {
        a += __shfl_xor(a, d);
        c += __shfl_xor(c, d);
      }
      if ((threadIdx.x & 63) == 0) {
        if (a) atomicAdd(&tot[q], a);
        if (c) atomicAdd(&pre[q], c);
      }
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 8) counts[threadIdx.x] = threadIdx.x < SDX_SEL_NCLASS ? tot[threadIdx.x] : 0;
  int cur[SDX_SEL_NCLASS];  // next free position of each class for this chunk (uniform)
  {
    int st = 0;
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
      cur[q] = st + pre[q];
      st += tot[q];
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int base = blockIdx.x * SDX_SEL_CHUNK;
  for (int r = 0; r < SDX_SEL_CHUNK; r += SEL_THREADS) {
    const int i = base + r + threadIdx.x;
    const int k = i < n ? sel_class(o, i) : -1;
    uint64_t m[SDX_SEL_NCLASS];
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q) {
      m[q] = __ballot(k == q);
      if (lane == 0) wcnt[wave][q] = __popcll(m[q]);
    }
    __syncthreads();
    if (k >= 0) {
      int pos = 0;
#pragma unroll
      for (int q = 0; q < SDX_SEL_NCLASS; ++q)
        if (q == k) {
          pos = cur[q] + __popcll(m[q] & lt);
          for (int w = 0; w < wave; ++w) pos += wcnt[w][q];
        }
      sel[pos] = i;
    }
#pragma unroll
    for (int q = 0; q < SDX_SEL_NCLASS; ++q)
      for (int w = 0; w < SEL_THREADS / 64; ++w) cur[q] += wcnt[w][q];
    __syncthreads();
  }
}

}  // namespace sdxl

extern "C" int sdx_select_lines(const sdx_lines_out* out, int32_t n, int32_t* sel_dev, int32_t* counts_dev,
                                int32_t* scratch_dev, void* hip_stream) {
  if (!out || n < 0 || !counts_dev) return sdx::set_error(SDX_EINVAL, "sdx_select_lines: bad arguments");
  hipStream_t st = (hipStream_t)hip_stream;
  if (n == 0) {
    const hipError_t e = hipMemsetAsync(counts_dev, 0, 8 * sizeof(int32_t), st);
    return e == hipSuccess ? SDX_OK : sdx::set_error(SDX_EHIP, "sdx_select_lines: memset failed");
  }
  if (!sel_dev || !scratch_dev || !out->kind_dev || !out->status_dev || !out->dlen_dev || !out->ms_ok_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_select_lines: null buffer");
  const int nchunk = (n + SDX_SEL_CHUNK - 1) / SDX_SEL_CHUNK;
  hipLaunchKernelGGL(sdxl::k_sel_count, dim3(nchunk), dim3(sdxl::SEL_THREADS), 0, st, *out, n, scratch_dev);
  hipLaunchKernelGGL(sdxl::k_sel_write, dim3(nchunk), dim3(sdxl::SEL_THREADS), 0, st, *out, n, nchunk,
                     (const int32_t*)scratch_dev, sel_dev, counts_dev);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_select_lines: ") + hipGetErrorString(e));
  return SDX_OK;
}

extern "C" int sdx_parse_lines(const sdx_lines* lines, const sdx_lines_out* out, void* hip_stream) {
  if (!lines || !out || lines->n < 0) return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: bad arguments");
  if (lines->n == 0) return SDX_OK;
  if (!lines->bytes_dev || !lines->offsets_dev || !out->kind_dev || !out->status_dev || !out->slot_dev ||
      !out->doff_dev || !out->dlen_dev || !out->npat_dev || !out->pat_id_dev || !out->pat_val_dev ||
      !out->cp_slot_dev || !out->ms_ok_dev || !out->clock_dev || !out->mcbitnum_dev || !out->mcflags_dev ||
      !out->meta_dev || !out->plen_dev)
    return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: null buffer");
  if (((uintptr_t)out->meta_dev & 15) != 0)
    return sdx::set_error(SDX_EINVAL, "sdx_parse_lines: meta_dev must be 16-byte aligned");
  const int per_block = 64 * sdxl::PW;
  const int grid = (lines->n + per_block - 1) / per_block;
  hipLaunchKernelGGL(sdxl::k_parse_lines, dim3(grid), dim3(per_block), 0, (hipStream_t)hip_stream, *lines, *out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("sdx_parse_lines: ") + hipGetErrorString(e));
  return SDX_OK;
}
