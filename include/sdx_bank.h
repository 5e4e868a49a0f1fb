/*
 * sdx_bank.h -- binary layout of a compiled SIGNALduino protocol bank.
 *
 * The bank is compiled on the host from protocols.json (the reference's
 * sd_protocols/protocols.json, loaded by sd_protocols/sd_protocols.py:30-41)
 * by pysignalduino_amd/bank.py into ONE contiguous blob that is uploaded to
 * HBM once per device and read (through L2/LDS) by every kernel.  All records
 * are naturally aligned C structs; the Python side mirrors them with numpy
 * dtypes (align=True) and checks sizeof() through sdx_layout_size().
 *
 * Record order inside each class table = JSON insertion order of the bank,
 * which is the reference's iteration order (get_keys, sd_protocols.py:49-52)
 * and therefore the result order.
 */
#ifndef SDX_BANK_H
#define SDX_BANK_H
#include <stdint.h>

#define SDX_BANK_MAGIC 0x4B4E4253u /* "SBNK" */
#define SDX_BANK_VERSION 17u
#define SDX_MAXSEARCH 16 /* longest start/sync/one/zero/float list (start of id 111 = 14) */
#define SDX_MAXUNIQ 4    /* distinct values inside one search list (bank max: 4) */
#define SDX_MAXPAT 10    /* P0..P9: pattern ids are single digits (device contract) */

/* one search list (start/sync/one/zero/float) = pattern_exists() argument,
 * pattern_utils.py:34-136, with its unique values (first-appearance order)
 * and their tolerances (calculate_tolerance, pattern_utils.py:15-26) */
typedef struct {
  /* hot part (one 64-byte line): what the lane filter reads per (message, protocol) */
  /* the test on the integer k of a normalised value k/10 (round(x/clock, 1)):
   * candidate  <=>  klo[u] <= k <= khi[u]  (exact; computed by bank.py _k_interval) */
  int32_t klo[SDX_MAXUNIQ], khi[SDX_MAXUNIQ];
  /* candidate ordering (stable sort by fp64 gap, pattern_utils.py:61-63): rank of k in the u16
   * table at ranks[rk_off[u] + k - klo[u]]; equal gaps share a rank */
  uint32_t rk_off[SDX_MAXUNIQ];
  uint8_t len;   /* search length; 0 = key absent/falsy */
  uint8_t nuniq; /* number of distinct values */
  uint8_t pad[6];
  uint64_t uidx_pk;            /* search position -> unique index, nibble i */
  /* cold part: the values themselves (the long-message variant's fp64 path) */
  double uval[SDX_MAXUNIQ];
  double utol[SDX_MAXUNIQ];
  uint8_t uidx[SDX_MAXSEARCH]; /* the same as uidx_pk, one byte per position */
} sdx_patspec;                 /* 144 bytes, 64-byte hot part first */

enum sdx_postdemo {
  SDX_PD_NONE = 0, SDX_PD_EM, SDX_PD_REVOLT, SDX_PD_FS20, SDX_PD_FHT80, SDX_PD_FHT80TF,
  SDX_PD_WS2000, SDX_PD_WS7035, SDX_PD_WS7053, SDX_PD_LENPREFIX
};

/* MU protocol = every id with 'clockabs' (message_unsynced.py:45) */
typedef struct {
  double clock;                         /* float(clockabs)  (:59) */
  uint8_t has_start, recon, dispatch_bin, remove_zero, active, never, res0, res1;
  sdx_patspec start, one, zero, flt;    /* (:67-141) */
  int32_t proto_index;                  /* index into the full bank (host: pid string) */
  int32_t length_min;                   /* regex {min,}  (:178) */
  int32_t length_max;                   /* chunk-count limit, INT32_MAX = none (:217) */
  int32_t width;                        /* len(one)  (:201-206) */
  int32_t pad_bits;                     /* paddingbits (:257) */
  int32_t postdemo;                     /* enum sdx_postdemo (:231-250) */
  int32_t mm_dfa;                       /* modulematch DFA index, -1 = none (:277) */
  int32_t mm_pre_state;                 /* DFA state after consuming the (constant) preamble */
  int32_t pre_off, pre_len, post_off, post_len; /* string heap (:271-274) */
  int32_t res2;
} sdx_mu_proto;

/* The MU lane filter's view of one protocol, packed into ONE 128-byte aligned record (the scalar
 * data cache then fetches a protocol's filter state with two line reads instead of ~10): flags,
 * clock and the four search lists with k bounds as int16 and rank offsets as uint16.  A list that
 * does not fit (more than 3 distinct values, |k| > 32767, rank offset > 65535) sets `full`, and the
 * filter reads sdx_mu_proto instead. */
typedef struct {
  uint32_t lohi[3];      /* unique value u: klo in the low 16 bits (two's complement), khi in the high 16 */
  uint32_t rk01;         /* rk_off[0] | rk_off[1] << 16 */
  uint32_t rk2_len_nu;   /* rk_off[2] | len << 16 | nuniq << 24 */
  uint32_t upk;          /* uidx_pk (search lists of <= 8 positions; start: see start_upk) */
} sdx_fspec;             /* 24 bytes */
typedef struct {
  double clock;          /* float(clockabs) */
  uint64_t start_upk;    /* uidx_pk of the start list (<= 16 positions) */
  uint32_t flags;        /* bit0 has_start, bit1 never, bit2 active, bit3 full */
  sdx_fspec spec[4];     /* start, one, zero, float */
  /* integer normalisation of round(P / clockabs, 1) (message_unsynced.py:64) for integral P:
   * k = round-half-even(10*|P| / clk_c) with floor(x / clk_c) == (x * clk_m) >> clk_sh for every
   * x < 2^30 (Granlund-Montgomery); exact ties (2r == clk_c) and non-integral P take the fp64 path */
  uint32_t clk_c;        /* |clockabs| when it is an integer in [1, 2^20) */
  uint32_t clk_m;        /* ceil(2^clk_sh / clk_c) */
  uint32_t clk_sh;       /* bits 0-7: shift (30 + ceil(log2 clk_c)); bit 8: valid; bit 9: clockabs < 0 */
} sdx_mu_filt;           /* 128 bytes */

/* the MS lane filter's view of one protocol (as sdx_mu_filt; spec = sync, one, zero, float) */
typedef struct {
  double pclock;         /* float(clockabs or 0) */
  uint64_t sync_upk;     /* uidx_pk of the sync list */
  uint32_t flags;        /* bit1 never, bit3 full */
  int32_t width, lmin_sync;
  sdx_fspec spec[4];
  uint32_t res;
} sdx_ms_filt;           /* 128 bytes */

/* MS protocol = every id with 'sync' (message_synced.py:79) */
typedef struct {
  double pclock;                        /* float(clockabs or 0)  (:83) */
  sdx_patspec key[4];                   /* sync, one, zero, float (:109) */
  int32_t proto_index;
  int32_t width;                        /* len(one) (:106-107) */
  int32_t lmin_sync;                    /* int(length_min or -1) (:152) */
  int32_t lir_min;                      /* length_in_range min, -1 none (helpers.py:144-154) */
  int32_t lir_max;                      /* length_in_range max, INT32_MAX none (helpers.py:157-164) */
  int32_t pad_bits, postdemo, pre_off, pre_len, post_off, post_len;
  uint8_t recon, never, res[2];
} sdx_ms_proto;

enum sdx_mc_method {
  SDX_MC_FUNKBUS = 1, SDX_MC_SAINLOGIC, SDX_MC_AS, SDX_MC_PLAIN, SDX_MC_RAW, SDX_MC_HMCRAW, SDX_MC_TFA,
  SDX_MC_GROTHE, SDX_MC_SOMFY
};

#define SDX_PID_NOT_INT ((int32_t)0x80000000)

/* MC protocol = every id with 'clockrange' (manchester.py:49-144); the unit entry (sdx_units) takes
 * one such record per call, built by the host for any protocol id */
typedef struct {
  double cr_lo, cr_hi;                  /* clockrange[0], clockrange[1] */
  int32_t proto_index;
  int32_t method;                       /* enum sdx_mc_method */
  int32_t lmin, lmax;                   /* parsed length_min / length_max */
  int32_t pre_off, pre_len;
  int32_t pid_num;                      /* int(pid) (Funkbus id test); SDX_PID_NOT_INT when int() raises */
  uint8_t has_lmin, has_lmax, lmax_is_str, invert, has_cr;
  uint8_t lir_noexist;                  /* length_in_range: protocol_exists(str(pid)) is False */
  uint8_t res[2];
} sdx_mc_proto;

/* MN protocol = every id with 'modulation' (signalduino/parser/mn.py:80) */
enum sdx_mn_method {
  SDX_MN_RAW = 0,        /* no 'method': the payload is the hex data (mn.py:121) */
  SDX_MN_LIGHTNING = 1,  /* helpers.py:223-280 ConvBresser_lightning */
  SDX_MN_5IN1 = 2,       /* helpers.py:382-425 ConvBresser_5in1 */
  SDX_MN_6IN1 = 3,       /* helpers.py:427-471 ConvBresser_6in1 */
  SDX_MN_7IN1 = 4,       /* helpers.py:473-523 ConvBresser_7in1 */
  SDX_MN_PCA301 = 5,     /* helpers.py:525-579 ConvPCA301 */
  SDX_MN_KOPP = 6,       /* helpers.py:581-628 ConvKoppFreeControl */
  SDX_MN_LACROSSE = 7,   /* helpers.py:630-716 ConvLaCrosse */
  SDX_MN_MISSING = 255   /* a 'method' the reference class does not define: protocol skipped (mn.py:171-173) */
};
#define SDX_MN_MAX 64    /* MN protocols in a bank (sdx_mn_batch.elig is a 64-bit mask) */
/* MN checksum tables (byte offsets inside the SDX_MNTAB_BYTES block at off_mntab) */
#define SDX_MNTAB_CRC1021 0     /* u16[256] */
#define SDX_MNTAB_CRC8005 512   /* u16[256] */
#define SDX_MNTAB_CRC31 1024    /* u8[256] */
#define SDX_MNTAB_LFSR8 1280    /* u16[16][16]: ConvBresser_lightning, key 0xABF9 */
#define SDX_MNTAB_LFSR21 1792   /* u16[42][16]: ConvBresser_7in1, key 0xBA95 */
#define SDX_MNTAB_BYTES 3136
typedef struct {
  int32_t proto_index;
  int32_t lir_min;       /* length_in_range on len(hex) (helpers.py:124-166): -1 = none */
  int32_t lir_max;       /* INT32_MAX = none */
  int32_t dfa;           /* regexMatch search DFA (re.search, mn.py:104-113), -1 = no regexMatch */
  int32_t method;        /* enum sdx_mn_method */
  int32_t pre_off, pre_len;  /* preamble (mn.py:176-177) in the string heap */
  int32_t dfa_slot;      /* distinct-regexMatch index (< 32): k_mn evaluates each pattern once per frame */
} sdx_mn_proto;          /* 32 bytes */

/* JSON fragments of one protocol for sdx_serialize_json (the MQTT publication of a DecodedMessage,
 * signalduino/mqtt.py:227-245: json.dumps(asdict(msg) minus raw, indent=4)), rendered on the host
 * with Python's json module into the string heap: pid = json.dumps(protocol_id); s1 = MU:
 * json.dumps(float(clockabs)) (meta.clock), MN: json.dumps(modulation); s2 = MN: json.dumps(rfmode). */
typedef struct {
  uint32_t pid_off, s1_off, s2_off;
  uint16_t pid_len, s1_len, s2_len, res;
} sdx_json_rec;          /* 20 bytes */

/* MU decode descriptor: the fields the compacted MU decode reads for one (message, protocol)
 * pair (message_unsynced.py:146-290), staged in LDS once per tile (the first SDX_MUDESC_LDS).
 * mm_on: 0 no modulematch; 1 LDS tables: st = mmtab[(mm_base + st) * 16 + digit] per hex digit,
 * then st = mmtab[17 * S + mm_post + st] for the postamble, accept on flags mmtab[16 * S + mm_base
 * + st] (ACC_NOW and DEAD are absorbing); 2 byte walk through the blob's t256 table; 3 the table
 * walk's outcome depends on the digit count only (bank.py _mm_length_interval, exact for <= 64
 * digits): accept iff res[0] <= digits <= res[1], no walk (the non-fast paths walk t256 as for 2). */
#define SDX_MUDESC_LDS 144
#define SDX_MMTAB_LDS 10240
typedef struct {
  uint8_t pre[16], post[2];             /* preamble / postamble bytes (longer ones: string heap) */
  uint8_t pre_len, post_len;
  uint8_t width, len_s, recon, dispatch_bin, remove_zero, postdemo, pad_bits, mm_on;
  uint16_t lmin, lmax;                  /* chunk-count limits, 65535 = none */
  uint16_t mm_base, mm_post;
  uint8_t pre_state, res[3];           /* mm_on 3: res[0..1] = accepted digit counts [lo, hi] */
} sdx_mu_desc;                          /* 40 bytes */

/* modulematch DFA (search semantics of re.search over the payload).
 * flags: bit0 = a match has been found (absorbing), bit1 = match if the payload
 * ends here ('$'), bit2 = dead (no match possible any more). */
typedef struct {
  int32_t nstates, start, trans_off, flags_off; /* into the DFA heaps (u16 class trans, u8 flags) */
  int32_t t256_off, res[3];                     /* u8 [nstates][256] byte-indexed transitions */
} sdx_dfa;

typedef struct {
  uint32_t magic, version;
  uint32_t n_proto, n_mu, n_ms, n_mc, n_dfa, n_class;
  uint32_t off_mu, off_ms, off_mc, off_dfa, off_cls, off_trans, off_flags, off_str;
  uint32_t total_bytes, off_t256;
  uint32_t off_order; /* u16 processing order: n_mu MU record indices (grouped by clock), then n_ms MS
                       * indices, then n_mu_groups + 1 MU group starts */
  uint32_t off_rank;  /* u16 candidate gap-rank tables (sdx_patspec.rk_off) */
  uint32_t off_mudesc;  /* sdx_mu_desc[n_mu] */
  uint32_t off_mmtab;   /* u8 modulematch tables for the MU decode (see sdx_mu_desc) */
  uint32_t mmtab_bytes; /* <= SDX_MMTAB_LDS, multiple of 16 */
  uint32_t mm_states;   /* S: hex[S][16] at 0, flags[S] at 16*S, post tables at 17*S */
  uint32_t n_mu_groups; /* MU clock groups: order[n_mu + n_ms + g] .. [+ g + 1] bound group g */
  uint32_t n_mn;        /* MN protocols (sdx_mn_proto[n_mn] at off_mn) */
  uint32_t off_mn;
  uint32_t off_json;    /* sdx_json_rec[n_mu + n_ms + n_mc + n_mn], class-major (MU, MS, MC, MN) */
  uint32_t off_mufilt;  /* sdx_mu_filt[n_mu], 128-byte aligned */
  uint32_t off_msfilt;  /* sdx_ms_filt[n_ms], 128-byte aligned */
  uint32_t off_mntab;   /* MN checksum tables (SDX_MNTAB_BYTES, bank.py mn_tables) */
} sdx_bank_hdr;

#endif
