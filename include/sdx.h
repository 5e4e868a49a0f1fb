/*
 * sdx.h -- C-ABI of the MI355X-native SIGNALduino MU/MS/MC demodulator.
 *
 * This is the drop-in boundary for the reference's demodulation entry points
 * (RFD-FHEM/PySignalduino):
 *   SDProtocols.demodulate(msg_data, msg_type)      sd_protocols/sd_protocols.py:60-74
 *   SDProtocols.demodulate_mu(msg_data, msg_type)   sd_protocols/message_unsynced.py:11-296
 *   SDProtocols.demodulate_ms(msg_data, msg_type)   sd_protocols/message_synced.py:10-243
 *   SDProtocols.demodulate_mc(msg_data, msg_type)   sd_protocols/sd_protocols.py:76-111
 *                                                   + manchester.py:49-144 ("fixed" mode)
 *   MNParser.parse(frame) per-protocol loop         signalduino/parser/mn.py:79-191
 *   SDProtocols.demodulate_mn / ConvBresser_* / ConvPCA301 / ConvKoppFreeControl / ConvLaCrosse
 *                                                   sd_protocols/sd_protocols.py:113-154, helpers.py:190-716
 * The Python host mirror (pysignalduino_amd/sd_protocols.py) binds these with
 * ctypes; INTEGRATION.md shows the binding.  All pointers named *_dev are
 * device (HBM) pointers owned by the caller; the library never allocates in a
 * launch function (graph-capturable) except inside sdx_bank_create.
 *
 * Error convention: every function returns 0 on success and a negative
 * SDX_E* code on failure (sdx_last_error() gives text).  No C++ exception
 * crosses the ABI.  Per-message outcomes (ok / reference raised / overflow)
 * are reported in the descriptor array, see sdx_desc below.
 */
#ifndef SDX_H
#define SDX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDX_ABI_VERSION 14

enum { SDX_OK = 0, SDX_EINVAL = -1, SDX_EHIP = -2, SDX_EBANK = -3, SDX_ECONTRACT = -4 };

enum sdx_kind { SDX_KIND_MU = 0, SDX_KIND_MS = 1, SDX_KIND_MC = 2, SDX_KIND_MN = 3 };

/* per-message status in sdx_desc.status */
enum sdx_status {
  SDX_ST_OK = 0,       /* results [rec_begin, rec_begin+n_rec) are the reference's list */
  SDX_ST_RAISED = 1,   /* the reference raises: raise_kind says which exception */
  SDX_ST_OVF_TILE = 2, /* on-chip result staging overflowed: re-run this message */
  SDX_ST_OVF_OUT = 3,  /* the caller's result/heap capacity overflowed: grow and re-run */
  SDX_ST_ABSENT = 0xFF /* ABI 11: an exchange overlay's descriptor that no re-run wrote (the caller fills an
                        * overlay's descriptors with 0xFF bytes before its re-run launches) */
};
/* sdx_desc.raise_kind (Python exception class the reference raises) */
enum sdx_raise { SDX_RAISE_NONE = 0, SDX_RAISE_INDEX = 1, SDX_RAISE_ATTRIBUTE = 2, SDX_RAISE_VALUE = 3,
                 SDX_RAISE_TYPE = 4, SDX_RAISE_ZERODIV = 5,
                 SDX_RAISE_CONTRACT = 6 /* not a reference outcome: the message exceeds a general-path limit
                                         * (SDX_GEN_*); the host reports it as outside the device contract */ };

typedef struct {
  uint32_t rec_begin; /* index of the first result record of this message */
  uint16_t n_rec;     /* number of results */
  uint8_t status;     /* enum sdx_status */
  uint8_t raise_kind; /* enum sdx_raise */
} sdx_desc;

typedef struct {
  uint32_t payload_off; /* byte offset of the payload (dmsg) in the heap */
  uint16_t payload_len;
  uint16_t proto;       /* record index inside the class table (bank order) */
  uint32_t bit_length;  /* meta.bit_length (MU/MS); 0 for MC */
  uint32_t msg;         /* message index (into the batch) */
} sdx_result;

/* One message's header fields packed into one 128-byte record (sdx_group_pulses writes them while it
 * reads the batch in message order; sdx_pulse_batch.mrec_dev).  A grouped launch visits its messages
 * in the grouped order, so read from the SoA arrays every field is its own scattered 32-64 B memory
 * sector per message; from the record they are one aligned line. */
typedef struct {
  int64_t off;          /* offsets[i] */
  int32_t len;          /* the message's length (len_dev[i], or offsets[i+1] - offsets[i]) */
  uint8_t npat;         /* npat[i] */
  int8_t cp_slot;       /* MS: cp_slot[i]; MU: -1 */
  uint8_t ms_ok;        /* MS: ms_ok[i]; MU: 0 */
  uint8_t res0;
  uint8_t pat_id[10];   /* pat_id[10 i, 10 i + 10) */
  uint8_t res1[6];
  double pat_val[10];   /* pat_val[10 i, 10 i + 10) (slots >= npat: 0) */
  uint8_t res2[16];
} sdx_msg_rec;          /* 128 bytes */

/* MU / MS batch: structure-of-arrays in HBM (see DESIGN.md "Data layout") */
typedef struct {
  const uint8_t* data_dev;     /* pulse-id characters, all messages concatenated */
  const int64_t* offsets_dev;  /* [n+1] message i = data[offsets[i], offsets[i+1]) */
  const uint8_t* npat_dev;     /* [n] number of P# patterns (<= 10) */
  const uint8_t* pat_id_dev;   /* [n*10] ASCII id digit of pattern slot k, dict order */
  const double* pat_val_dev;   /* [n*10] float(P#) */
  const int8_t* cp_slot_dev;   /* [n] MS: slot of CP, -1 = CP not a pattern (NULL for MU) */
  const uint8_t* ms_ok_dev;    /* [n] MS: CP/SP/R string gates passed (NULL for MU) */
  const int32_t* len_dev;      /* optional [n] message lengths: message i = data[offsets[i], +len[i])
                                * (slot layout of sdx_parse_lines); NULL = offsets[i+1] - offsets[i] */
  const int32_t* sel_dev;      /* optional [n_sel] subset of message indices to run, NULL = all */
  int32_t n;                   /* messages in the batch */
  int32_t n_sel;               /* entries in sel_dev (ignored when sel_dev == NULL) */
  const sdx_msg_rec* mrec_dev; /* optional [n]: the header fields of every message the launch visits,
                                * as sdx_group_pulses wrote them (the short MU/MS variant reads them
                                * from here; the SoA arrays must still be given); NULL = SoA only */
} sdx_pulse_batch;

/* MC batch */
typedef struct {
  const uint8_t* hex_dev;      /* hex characters (D=) of all frames concatenated; readable 8 bytes
                                * past every frame's end (k_mc stages frames with aligned 8-byte loads) */
  const int64_t* offsets_dev;  /* [n+1] */
  const int32_t* clock_dev;    /* [n] C= */
  const int32_t* mcbitnum_dev; /* [n] L= */
  const uint8_t* flags_dev;    /* [n] bit0: message type 'Mc', bit1: version starts 'V 3.2.' */
  const int32_t* len_dev;      /* optional [n] frame lengths (as sdx_pulse_batch.len_dev) */
  const int32_t* sel_dev;
  int32_t n, n_sel;
  const int16_t* only_dev;     /* optional [n]: evaluate only MC protocol only[i] (table index; -1 = every
                                * protocol) -- demodulate_mc(msg_data) with a protocol_id (sd_protocols.py:79) */
  int32_t max_hex;             /* ABI 13, optional: an upper bound on the length (hex characters) of every
                                * frame run, 0 = unknown.  sdx_demod_mc launches its 65..128-character
                                * variant only when max_hex is 0 or > SDX_MC_SHORT_HEX; a frame longer
                                * than a bound of <= SDX_MC_SHORT_HEX gets SDX_ST_OVF_TILE (cursor[2]
                                * bit 1), as frames past SDX_MC_HEX_MAX do */
  int32_t res;
} sdx_mc_batch;
#define SDX_MC_SHORT_HEX 64    /* frames up to this length run in sdx_demod_mc's 4-word variant */

/* MN (FSK) batch: the hex characters of each frame (MN_PATTERN group 2, parser/mn.py:17) */
typedef struct {
  const uint8_t* hex_dev;      /* hex characters of all frames; readable 8 bytes past every frame's end
                                * (k_mn stages frames with aligned 4-byte loads) */
  const int64_t* offsets_dev;  /* [n+1] frame i = hex[offsets[i], offsets[i+1]) (or + len[i]) */
  const int32_t* len_dev;      /* optional [n] frame lengths (as sdx_pulse_batch.len_dev) */
  const int32_t* sel_dev;      /* optional [n_sel] subset of frame indices to run, NULL = all */
  int32_t n, n_sel;
  uint64_t elig;               /* parser mode: bit k = MN protocol k (bank order) passes the rfmode filter
                                * (parser/mn.py:83-93; the host folds MNParser.rfmode in) */
  int32_t method;              /* -1: parser mode (MNParser.parse, results = bank protocols in order,
                                * payload = preamble + decoded, a failed method gives "[]");
                                * >= 1: method mode, enum sdx_mn_method: the method alone per frame
                                * (SDProtocols.ConvX(msg_data)), 0 or 1 result with its payload */
  int32_t res;
} sdx_mn_batch;

/* output buffers (caller-owned, device) */
typedef struct {
  sdx_desc* desc_dev;          /* [n] */
  sdx_result* rec_dev;         /* [rec_cap] */
  uint8_t* heap_dev;           /* [heap_cap] */
  uint32_t* cursor_dev;        /* [4] zeroed by the caller before the first launch: rec, heap, ovf,
                                * spill regions handed out (including refused ones past work_cap) */
  uint32_t rec_cap, heap_cap;
  uint8_t* work_dev;           /* optional device workspace (MU/MS short variant, NULL = none), 256-B
                                * aligned: spill regions of result-heavy tiles (112 KB each, see
                                * sdx_pulses_work_bytes); without it a tile whose results overflow
                                * LDS is re-run (ST_OVF_TILE) */
  uint64_t work_cap;           /* bytes at work_dev (< 4 GiB - 112 KB: spill offsets are 32-bit) */
  /* ABI 12, optional (NULL = none): the exchange's view of the results, written by the flushes of
   * sdx_demod_pulses / _long and sdx_demod_mc while the payloads are still on chip, so that
   * sdx_exchange_count / _pack need not classify every payload again:
   *   wire_dev[n]        per message: (payload bytes << 32) | wire payload bytes of its records (0 for
   *                      a message without results; written with its descriptor)
   *   xrec_dev[rec_cap]  per record (same index as rec_dev): SDX_XREC_NIB | preamble length << 16 |
   *                      hex digit count when the payload is preamble + uppercase hex + postamble of
   *                      its protocol (the nibble form), 0 otherwise */
  uint64_t* wire_dev;
  uint32_t* xrec_dev;
} sdx_out;
#define SDX_XREC_NIB 0x80000000u

typedef struct sdx_bank sdx_bank;

int sdx_abi_version(void);
const char* sdx_last_error(void);
/* sha256 prefix of the sources and flags the library was built from (pysignalduino_amd/build.py
 * source_hash): a caller can check that it loaded the library of the tree it runs in */
const char* sdx_source_hash(void);
/* sizeof() of the bank records, for host layout checks: 0 hdr, 1 patspec, 2 mu, 3 ms, 4 mc, 5 result, 6 desc,
 * 7 mu_desc */
int sdx_layout_size(int which);

/* stream-ordered byte copy / fill on the caller's stream (hipMemcpyAsync with hipMemcpyDefault,
 * hipMemsetAsync): the streaming pipeline's per-chunk H2D / D2H transfers and buffer resets, without a
 * framework's per-call dispatch.  Host buffers must be pinned for the copy to be asynchronous. */
int sdx_copy_async(void* dst, const void* src, size_t nbytes, void* hip_stream);
/* the same with the direction given (a hipMemcpyKind: 1 host->device, 2 device->host, 3 device->device,
 * 4 inferred as sdx_copy_async does): the HIP runtime picks its copy engine by it */
int sdx_copy_async_kind(void* dst, const void* src, size_t nbytes, int kind, void* hip_stream);
/* a device -> pinned-host (or any device-accessible) copy by a kernel of nwg 256-thread workgroups:
 * occupies nwg CU slots for the transfer instead of the runtime's blit kernel on every CU */
int sdx_copy_async_narrow(void* dst, const void* src, size_t nbytes, int nwg, void* hip_stream);
int sdx_fill_async(void* dst, int value, size_t nbytes, void* hip_stream);

/* bank: compiled by pysignalduino_amd/bank.py (protocols.json -> blob) and uploaded once per device */
int sdx_bank_create(const void* blob, size_t nbytes, int device, sdx_bank** out);
int sdx_bank_destroy(sdx_bank* bank);
const void* sdx_bank_device_ptr(const sdx_bank* bank);

/* MU/MS demodulation of a batch (or of batch->sel_dev, in that order): results appended to out */
int sdx_demod_pulses(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, const sdx_out* out,
                     void* hip_stream);
/* out->work_cap for `spill_tiles` result-heavy tiles (112 KB each; a tile of 64 messages spills when
 * its results exceed 512 records / 10 KB of payload / 768 matches in LDS) */
size_t sdx_pulses_work_bytes(int spill_tiles);
/* Message grouping (sdx_group.hip): order_dev[0, n) = the batch's messages (or batch->sel_dev's) in
 * the order of a per-message key -- which of the first 32 protocols (bank order) the message passes
 * the candidate-interval test of -- by a device radix sort.  sdx_demod_pulses on that order (as
 * sel_dev) gives the same results with fewer instructions (tiles of messages that survive the same
 * protocols).  work_dev: sdx_group_work_bytes(n) bytes.  Worth it from a few thousand messages. */
size_t sdx_group_work_bytes(int n);
/* mrec_dev: optional [batch->n] records (sdx_msg_rec) written for every message grouped -- pass them
 * as the launch's batch->mrec_dev; NULL = none written */
int sdx_group_pulses(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, int32_t* order_dev,
                     sdx_msg_rec* mrec_dev, void* work_dev, size_t work_cap, void* hip_stream);
#define SDX_GROUP_MIN 4096  /* batches from this size are grouped by the host wrappers */
/* ABI 14: a mixed step's MU and MS groupings (the results of two sdx_group_pulses calls) with both
 * sorts' passes in the same launches: 13 launches instead of 26 */
typedef struct sdx_group_job {
  const sdx_pulse_batch* batch;
  int32_t* order_dev;
  sdx_msg_rec* mrec_dev;  /* optional */
  void* work_dev;
  size_t work_cap;
} sdx_group_job;
int sdx_group_step(const sdx_bank* bank, const sdx_group_job* mu, const sdx_group_job* ms, void* hip_stream);
/* same, for messages of 257..4096 pulses (4 messages per workgroup tile) */
int sdx_demod_pulses_long(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, const sdx_out* out,
                          void* hip_stream);
/* MC "fixed" chain: every frame x every clockrange protocol.  Frames of more than SDX_MC_HEX_MAX
 * characters get status SDX_ST_OVF_TILE (cursor[2] bit 1): run them with sdx_demod_mc_general */
int sdx_demod_mc(const sdx_bank* bank, const sdx_mc_batch* batch, const sdx_out* out, void* hip_stream);
/* ABI 14: one mixed step -- the MU launch, the MS launch and the MC launch of a step, each optional
 * (NULL batch = none) -- as ONE kernel (k_step): workgroups [0, MU tiles) run MU's tiles, then MS's,
 * then MC's frames, so each kind's tiles take the CU slots the previous kind's last tiles free instead
 * of waiting for its whole launch to end.  Results are those of sdx_demod_pulses(MU),
 * sdx_demod_pulses(MS) and sdx_demod_mc on the same stream in that order (record order inside a launch
 * is tile order either way).  Parts the fused kernel does not cover (an MS batch with mrec_dev, MC frames
 * that may exceed SDX_MC_SHORT_HEX characters) run their own launches after it on the stream. */
typedef struct sdx_step {
  const sdx_pulse_batch* mu;
  const sdx_out* mu_out;
  const sdx_pulse_batch* ms;
  const sdx_out* ms_out;
  const sdx_mc_batch* mc;
  const sdx_out* mc_out;
} sdx_step;
int sdx_demod_step(const sdx_bank* bank, const sdx_step* step, void* hip_stream);
/* MN (FSK): every frame x every 'modulation' protocol (parser mode) or one method (method mode).
 * Frames must hold hex digits only ([0-9A-Fa-f]; the front end guarantees [0-9A-F]) and at most
 * SDX_MN_HEX_MAX of them.  sdx_result.proto = MN table index (parser mode) / the method (method mode). */
int sdx_demod_mn(const sdx_bank* bank, const sdx_mn_batch* batch, const sdx_out* out, void* hip_stream);

/* ---- general path (messages outside the short / long kernels' contract) ------------------------
 * MU/MS messages the fixed-layout kernels do not take: pattern ids of more than one digit (the
 * reference keys patterns by str(int(key[1:])) for any "P<digits>" key, message_unsynced.py:28-35,
 * message_synced.py:50-57 -- "P10" is pattern "10", and pattern_exists concatenates such strings,
 * pattern_utils.py:120-130), more than 10 patterns, and more than SDX_LONG_MAX pulses.  The
 * reference's string semantics run as they are: candidate targets are character strings, MU's
 * re.finditer over (?:start)((?:u1|u2|..){length_min,}(?:e1|..)?) is emulated with Python sre's
 * backtracking order, chunks are sliced by characters.  A wave walks a chunk of the bank (a few
 * protocols in bank order) for one message, the chunks of a message run on separate waves (the
 * first raise in bank order decides, as in the reference); every result list is counted, reserved
 * (one atomic pair per message) and written in a second pass.  out->work_dev must hold
 * sdx_general_work_bytes(...) bytes.  Limits (status SDX_ST_RAISED + SDX_RAISE_CONTRACT when
 * exceeded): SDX_GEN_MAXPAT patterns of <= 15 digits, target strings of <= SDX_GEN_STRMAX
 * characters, length_min <= SDX_GEN_REPMAX, 2^22 sre steps per repetition match, payloads of
 * <= 65535 bytes. */
#define SDX_GEN_MAXPAT 16
#define SDX_GEN_IDSTR 16    /* bytes per pattern id: [0] = length (1..15), [1..15] its digits */
#define SDX_GEN_STRMAX 64
#define SDX_GEN_REPMAX 128
typedef struct {
  const uint8_t* data_dev;     /* pulse-id characters, all messages concatenated */
  const int64_t* offsets_dev;  /* [n+1] message i = data[offsets[i], offsets[i+1]) */
  const uint8_t* npat_dev;     /* [n] patterns (<= SDX_GEN_MAXPAT) */
  const uint8_t* pat_ids_dev;  /* [n * SDX_GEN_MAXPAT * SDX_GEN_IDSTR] id string of pattern slot k, dict order */
  const double* pat_val_dev;   /* [n * SDX_GEN_MAXPAT] float(P#) */
  const int8_t* cp_slot_dev;   /* [n] MS: slot of str(int(CP)) (NULL for MU) */
  const uint8_t* ms_ok_dev;    /* [n] MS: string gates passed and CP names a pattern (NULL for MU) */
  const int32_t* sel_dev;      /* optional [n_sel] subset to run, NULL = all */
  int32_t n, n_sel;
  const int32_t* len_dev;      /* optional [n] lengths: message i = data[offsets[i], +len[i]) (slot layout) */
  int64_t work_stride;         /* > 0: the j-th message run takes its region at j * work_stride
                                * (>= 5 * (max_len + 512)); 0: regions by offsets (5 * offsets[i] + 2560 * i) */
  int32_t max_len;             /* HARD BOUND: the longest message run (characters); per-wave scratch, regions and LDS
                                * are sized by it -- a message longer than max_len is not walked (SDX_RAISE_CONTRACT) */
  int32_t res;
} sdx_general_batch;

/* workspace of a general-path launch of n messages (sel'd or not): a head (work queue counters, the
 * per (message, chunk of protocols) table, per-wave scratch) and the per-message regions */
uint64_t sdx_general_work_bytes(const sdx_bank* bank, int kind, int64_t total_chars, int32_t n, int32_t max_len,
                                int64_t work_stride);
int sdx_demod_pulses_general(const sdx_bank* bank, int kind, const sdx_general_batch* batch, const sdx_out* out,
                             void* hip_stream);
/* MC frames of any length (the "fixed" chain of sdx_demod_mc without its SDX_MC_HEX_MAX limit): lane =
 * frame, the frame's bits in out->work_dev (sdx_mc_general_work_bytes(frames run, max_hex) bytes),
 * results counted, reserved and written in a second pass.  Payloads of <= 65535 bytes. */
uint64_t sdx_mc_general_work_bytes(int32_t n, int32_t max_hex);
int sdx_demod_mc_general(const sdx_bank* bank, const sdx_mc_batch* batch, int32_t max_hex, const sdx_out* out,
                         void* hip_stream);

/* ---- wire-line front end ------------------------------------------------------
 * Raw firmware lines, byte for byte as the transport receives them (the reference decodes them
 * latin-1, signalduino/transport.py:123).  One launch runs, per line, what
 * SignalParser.parse_line does before demodulation (signalduino/parser/__init__.py:37-49):
 * strip + STX/ETX framing (parser/base.py:188-206), decompress_payload (base.py:13-186), routing
 * by payload[:2].upper(), the MU validity regex (parser/mu.py:48), _parse_to_dict and the "D"
 * check (mu.py:82-94, ms.py:65-78), and the MC header validation (parser/mc.py:37-155).  The
 * outputs of a line form message i of an sdx_pulse_batch (MU/MS) or sdx_mc_batch (MC) in slot
 * layout (len_dev set): no host repacking.  MN lines (parser/mn.py:31-51): MN_PATTERN is checked,
 * the hex characters (without the 'Y' prefix) become frame i of an sdx_mn_batch, R and A are
 * handed back raw in meta_dev (R at bytes 0-15, A at 16-31). */
enum sdx_line_kind { SDX_LINE_NONE = 0, SDX_LINE_MU = 1, SDX_LINE_MS = 2, SDX_LINE_MC = 3, SDX_LINE_MN = 4 };
enum sdx_line_status {
  SDX_LS_OK = 0,          /* routed to kind, ready for demodulation */
  SDX_LS_NOFRAME = 1,     /* extract_payload() returned None: ignored */
  SDX_LS_NOPARSER = 2,    /* no parser for the message type: ignored */
  SDX_LS_INVALID = 3,     /* the parser rejects the line (MU regex, MC header, MC hex, R/F): ignored */
  SDX_LS_NODATA = 4,      /* no D field: ignored */
  SDX_LS_UNSUPPORTED = 5, /* outside the device contract (e.g. P# values outside the exact float() subset,
                           * bytes >= 0x80 after decompression): the caller must not guess */
  SDX_LS_RAISES = 6,      /* handed to the demodulator, which raises (caught by the parser): no results
                           * (MC: int(C) / int(L) of a hex-lettered value) */
  SDX_LS_GENERAL = 7      /* an MU/MS line the fixed-layout kernels do not take (a multi-digit pattern id,
                           * more than SDX_LONG_MAX pulses): D, meta and doff/dlen are written as for
                           * SDX_LS_OK; sdx_lines_general builds its general-path batch */
};

typedef struct {
  const uint8_t* bytes_dev;    /* all lines concatenated; 8-byte aligned and readable 16 bytes past
                                * offsets[n] (the kernel reads whole aligned 8-byte words) */
  const int64_t* offsets_dev;  /* [n+1] line i = bytes[offsets[i], offsets[i+1]) */
  int32_t n;
} sdx_lines;

typedef struct {
  uint8_t* kind_dev;           /* [n] enum sdx_line_kind */
  uint8_t* status_dev;         /* [n] enum sdx_line_status */
  uint8_t* slot_dev;           /* [3 * offsets[n] + 16], 8-byte aligned; per-line slots: line i owns
                                * [3*offsets[i], 3*offsets[i+1]) */
  int64_t* doff_dev;           /* [n] start of the D (MU/MS) or hex (MC) characters in slot_dev */
  int32_t* dlen_dev;           /* [n] their length */
  uint8_t* npat_dev;           /* [n]   MU/MS: patterns (see sdx_pulse_batch) */
  uint8_t* pat_id_dev;         /* [n*10] */
  double* pat_val_dev;         /* [n*10] */
  int8_t* cp_slot_dev;         /* [n]   MS */
  uint8_t* ms_ok_dev;          /* [n]   MS */
  int32_t* clock_dev;          /* [n]   MC: int(C) */
  int32_t* mcbitnum_dev;       /* [n]   MC: int(L) */
  uint8_t* mcflags_dev;        /* [n]   MC: sdx_mc_batch flags (MCParser: type "MC", no version) */
  uint8_t* meta_dev;           /* [n*32] raw R (bytes 0-14, length at 15, 255 = absent; longer
                                * values make the line SDX_LS_UNSUPPORTED) and
                                * F (16-30, length at 31) strings, for meta.rssi / frame.rssi / frame.freq_afc */
  int32_t* plen_dev;           /* [n] decompressed lines: payload length at slot_dev + 3*offsets[i] (RawFrame.line);
                                * -1 = not decompressed (the payload is the stripped line between STX and ETX) */
} sdx_lines_out;

/* parse a batch of lines into out (device buffers, caller-owned; no allocation, no sync).  Lines
 * (MU/MS lines with multi-digit pattern ids or more than SDX_LONG_MAX pulses: SDX_LS_GENERAL) are
 * reported SDX_LS_UNSUPPORTED.  kind/status/doff/plen are written for every line; the other
 * fields only where they mean something: dlen and meta for SDX_LS_OK lines, the pattern fields
 * (npat, pat_id/pat_val[0..npat)) for OK MU/MS lines, cp_slot/ms_ok for OK MS lines, clock/
 * mcbitnum/mcflags for OK MC lines, and plen plus the slot payload for OK decompressed lines.
 * meta_dev must be 16-byte aligned; bytes_dev and slot_dev 8-byte aligned. */
int sdx_parse_lines(const sdx_lines* lines, const sdx_lines_out* out, void* hip_stream);

/* The general-path batch of a parsed batch's SDX_LS_GENERAL lines: for the j-th entry of sel_dev
 * (line i) the line's _parse_to_dict / _patterns fields in the sdx_general_batch layout --
 * offsets[j] = doff[i], len[j] = dlen[i] (the D characters in slot_dev), the pattern ids as strings
 * (str(int(key[1:]))), float(P#) values, MS cp_slot / ms_ok.  A line found outside the general
 * path's contract (an id of more than 15 digits, more than SDX_GEN_MAXPAT patterns) gets
 * status_dev[i] = SDX_LS_UNSUPPORTED and npat[j] = 0.  Run the result with
 * sdx_demod_pulses_general(data_dev = slot_dev, sel_dev = NULL, n = n_sel). */
typedef struct {
  int64_t* offsets_dev;        /* [n_sel] */
  int32_t* len_dev;            /* [n_sel] */
  uint8_t* npat_dev;           /* [n_sel] */
  uint8_t* pat_ids_dev;        /* [n_sel * SDX_GEN_MAXPAT * SDX_GEN_IDSTR] */
  double* pat_val_dev;         /* [n_sel * SDX_GEN_MAXPAT] */
  int8_t* cp_slot_dev;         /* [n_sel] */
  uint8_t* ms_ok_dev;          /* [n_sel] */
} sdx_lines_general_out;

int sdx_lines_general(const sdx_lines* lines, const sdx_lines_out* out, const int32_t* sel_dev, int32_t n_sel,
                      const sdx_lines_general_out* gen, void* hip_stream);

/* ---- publish-ready JSON ------------------------------------------------------
 * The MQTT publication of a DecodedMessage, MqttPublisher._message_to_json (signalduino/mqtt.py:
 * 227-245): json.dumps(asdict(message) minus "raw", indent=4), i.e.
 *   {"protocol_id": ..., "payload": ..., "metadata": {...}} with Python's separators, indentation,
 *   float repr and ensure_ascii escapes,
 * built on the device from one demodulation launch's outputs and the front end's per-line fields
 * (meta.rssi = the raw R string for MU/MS, meta.clock = float(clockabs) / abs(P[CP]); MC: protocol_id,
 * rssi/freq_afc null; MN: calc_rssi(R), round(26000000/16384*A/1000, 0), modulation, rfmode).
 * first_only = 1 gives the one message per line the controller publishes (decoded[0],
 * signalduino/controller.py:254-257); 0 gives one JSON text per result record; 2 (ABI 11) is 1 but
 * SPARSE: off/len are written only for the lines that get a text, so the launches of all kinds can
 * share one json_dev / off_dev / len_dev / cursor (a line belongs to one kind; the caller zeroes len). */
typedef struct {
  int32_t kind;                /* enum sdx_kind of the demodulation launch */
  int32_t first_only;
  const sdx_desc* desc_dev;    /* [n] the launch's descriptors (indexed by line) */
  const sdx_result* rec_dev;   /* its result records ... */
  const uint32_t* cursor_dev;  /* ... and its cursor: cursor[0] = record count (read on the device) */
  const uint8_t* heap_dev;     /* its payload heap */
  const uint8_t* meta_dev;     /* sdx_lines_out.meta_dev [n*32] */
  const double* pat_val_dev;   /* sdx_lines_out.pat_val_dev [n*10] (MS meta.clock) */
  const int8_t* cp_slot_dev;   /* sdx_lines_out.cp_slot_dev [n] */
  int32_t n;                   /* lines */
  int32_t rec_max;             /* first_only = 0: capacity of the record-indexed outputs */
} sdx_json_in;

typedef struct {
  uint8_t* json_dev;           /* JSON texts (ASCII), concatenated */
  uint32_t* off_dev;           /* [n] (first_only) or [rec_max]: offset of the text in json_dev */
  uint32_t* len_dev;           /* its length, 0 = no text (no result) */
  uint32_t* cursor_dev;        /* [2] zeroed by the caller: bytes used, overflow flag (grow json_cap, re-run) */
  uint32_t json_cap;
  uint32_t res;
} sdx_json_out;

int sdx_serialize_json(const sdx_bank* bank, const sdx_json_in* in, const sdx_json_out* out, void* hip_stream);

/* ---- unit-level entry ------------------------------------------------------------------------
 * The reference's helper methods that its own unit tests call on SDProtocols, evaluated on n
 * independent inputs in one launch (lane = item), with the device code the demodulation kernels
 * run.  Replaces, per op:
 *   SDX_UNIT_POSTDEMO   SDProtocols.postDemo_EM/_Revolt/_FS20/_FHT80/_FHT80TF/_WS2000/_WS7035/
 *                       _WS7053/_lengtnPrefix(name, bit_msg_array)   postdemodulation.py:27-730
 *                       in: the bits as bytes 0/1; arg: enum sdx_postdemo (sdx_bank.h).
 *                       proto 0: (1, payload bits as bytes 0/1); proto 1: (0, None);
 *                       RAISED ValueError: int('', 2).
 *   SDX_UNIT_HEX2BIN    SDProtocols.hex_to_bin_str(hex_string)      helpers.py:168-188, and with
 *                       arg = 1 _convert_mc_hex_to_bits's polarity translate first
 *                       (manchester.py:18-47).  in: the string's bytes; proto 0: payload '0'/'1';
 *                       proto 1: None.
 *   SDX_UNIT_BIN2HEX    SDProtocols.bin_str_2_hex_str(num)          helpers.py:28-64.
 *                       proto 0: payload (hex); proto 1: None.
 *   SDX_UNIT_MC2DMC     SDProtocols.mc2dmc(bit_data)                helpers.py:6-26 (ASCII input).
 *   SDX_UNIT_PEXISTS    pattern_utils.pattern_exists(search, patterns, raw_data)  pattern_utils.py:34-136.
 *                       in: [npat][npat id lengths][id bytes][raw_data]; val: the search values
 *                       then the pattern values (fp64, dict order); arg: number of search values
 *                       (<= SDX_UNIT_PX_SEARCH; npat <= SDX_UNIT_PX_PAT).  proto 0: the target
 *                       string; proto 1: -1.
 *   SDX_UNIT_MC_METHOD  SDProtocols.mcBit2Funkbus/Sainlogic/AS/Hideki/Maverick/OSV1/OSV2o3/OSPIR/
 *                       TFA/Grothe/SomfyRTS, mcRaw, mcraw(name, bit_data, protocol_id, mcbitnum)
 *                       manchester.py:207-795, helpers.py:90-122.  in: bit_data ('0'/'1',
 *                       <= SDX_UNIT_MC_BITS); arg: mcbitnum; mcrec_dev[i]: the sdx_mc_proto of
 *                       (protocol_id, method) (pysignalduino_amd/bank.py mc_record).  proto 0:
 *                       (1, payload), bit_length = payload kind (2: a Python list repr); proto k > 0:
 *                       (-1, text k) of the McWhy codes (csrc/sdx_mc.h), bit_length = its argument;
 *                       RAISED TypeError / ValueError where the reference raises.
 * Item i: desc[i] = {rec_begin i, n_rec 1 (0 when RAISED), status, raise_kind}, rec[i] = {payload at
 * heap[out_off[i]..], payload_len, proto (above), bit_length, msg i}; rec_cap >= n. */
enum sdx_unit_op { SDX_UNIT_POSTDEMO = 1, SDX_UNIT_HEX2BIN = 2, SDX_UNIT_BIN2HEX = 3, SDX_UNIT_MC2DMC = 4,
                   SDX_UNIT_PEXISTS = 5, SDX_UNIT_MC_METHOD = 6 };
#define SDX_UNIT_MC_BITS 512
#define SDX_UNIT_PX_SEARCH 32
#define SDX_UNIT_PX_PAT 16

typedef struct {
  int32_t op;                  /* enum sdx_unit_op */
  int32_t n;                   /* items */
  const uint8_t* in_dev;       /* item i's input: in[in_off[i], in_off[i+1]) */
  const int64_t* in_off_dev;   /* [n+1] */
  const int32_t* arg_dev;      /* [n] per-item argument (see above); NULL = 0 */
  const double* val_dev;       /* SDX_UNIT_PEXISTS: values of item i from val[val_off[i]] */
  const int64_t* val_off_dev;  /* SDX_UNIT_PEXISTS: [n+1] */
  const void* mcrec_dev;       /* SDX_UNIT_MC_METHOD: [n] sdx_mc_proto */
  const int64_t* out_off_dev;  /* [n+1] item i writes its payload to heap[out_off[i], out_off[i+1]) */
} sdx_unit_batch;

int sdx_units(const sdx_unit_batch* batch, const sdx_out* out, void* hip_stream);

/* ---- multi-GPU exchange (BASELINE config 5) --------------------------------------
 * The all-gather of decoded dmsg buffers (pysignalduino_amd/dist.py) moves a WIRE form of each
 * demodulation launch, per rank and in message order (the canonical order: the same bytes whether
 * the stream ran sharded or not):
 *   msg section   uint32 per message: n_rec | status << 16 | raise_kind << 24  (sdx_desc minus rec_begin)
 *   rec section   sdx_wire_rec per record                                      (sdx_result minus payload_off, msg)
 *   heap section  the payloads in record order; a payload that is its protocol's preamble + uppercase
 *                 hex digits + postamble (the bank's affixes; proto bit 15 = SDX_WIRE_NIB) travels as
 *                 its digits packed two per byte (high nibble first, an odd last digit in a high
 *                 nibble), any other payload as its bytes (ABI 11, wire v3)
 * rec_begin, payload_off, msg and the affixes are rebuilt by the receiver (sdx_exchange_unpack).
 * A rank's send buffer holds, for launch 0, 1, ..., K-1 in turn, its msg, rec and heap sections, each
 * zero-padded to 16 bytes -- a layout that follows from the counts alone (dist.py _layout).
 * Sender: sdx_exchange_count (device counts per launch + the layout), then sdx_exchange_pack into the
 * send buffer, both without a host round trip; the host needs the counts only to size the collective.
 * RE-RUNS (ABI 11): a launch part may name an OVERLAY part (alt = 1 + its index in the same array,
 * aux = 1 on the overlay): the outputs of the launches that re-ran the launch's overflowed messages,
 * over the same n_msgs, with every descriptor the re-runs did not write left at SDX_ST_ABSENT.  Message
 * m is taken from the LAST overlay along the chain (an overlay may name the next) whose descriptor of m is
 * present (at most 8 overlays per launch).
 * An aux part has no sections of its own (its counts are 0).
 * A message whose (resolved) status is an overflow, or whose descriptor / records lie outside what its
 * launch wrote (cursor clamped to the capacities), is counted in counts[3] ("bad") and shipped with
 * n_rec 0 and status SDX_ST_OVF_OUT: the caller re-runs it (into an overlay) before exchanging. */
#define SDX_XCHG_MAX_RANKS 32
#define SDX_XCHG_MAX_PARTS 16  /* launches + overlays per exchange */
#define SDX_XCHG_COUNTS 8      /* u32 counts per part: messages, records, wire payload bytes, bad, payload bytes, 0, 0, 0 */
#define SDX_WIRE_NIB 0x8000u   /* sdx_wire_rec.proto: the payload travels in the nibble form */
typedef struct {
  uint16_t proto;              /* record index in its class table | SDX_WIRE_NIB */
  uint16_t payload_len;        /* the payload's length (not its wire length) */
  uint32_t bit_length;
} sdx_wire_rec;

typedef struct {
  const uint8_t* desc_dev;     /* sdx_desc[n_msgs] of one demodulation launch */
  const uint8_t* rec_dev;      /* its sdx_result records */
  const uint8_t* heap_dev;     /* its payload heap */
  const uint32_t* cursor_dev;  /* its cursor: [0] records, [1] heap bytes written (clamped to rec_cap / heap_cap) */
  uint32_t n_msgs, rec_cap, heap_cap;
  uint8_t kind;                /* enum sdx_kind of the launch (its protocols' affixes); 0xFF: raw payloads only */
  uint8_t alt;                 /* 0, or 1 + index (in the same array) of this launch's overlay part */
  uint8_t aux;                 /* 1: this part is an overlay */
  uint8_t res;
  const uint64_t* wire_dev;    /* ABI 12, optional: the launch's sdx_out.wire_dev / xrec_dev (written by its
                                * kernels): messages with status OK are counted and packed from them */
  const uint32_t* xrec_dev;
} sdx_xchg_part;

/* workspace of count + pack (kept between the two: 12 B per message + block sums + a 256-byte head);
 * 256-byte aligned and ZEROED once at allocation (the kernels leave their counters at zero; any layout
 * of up to SDX_XCHG_MAX_PARTS parts may reuse one workspace of sufficient size) */
uint64_t sdx_exchange_work_bytes(const uint32_t* n_msgs, int k);
/* send buffer capacity for any outcome of the launches (from their and their overlays' capacities) */
uint64_t sdx_exchange_send_bytes(const sdx_xchg_part* parts, int k);
/* counts_dev[SDX_XCHG_COUNTS * i + 0..4] = messages, records, wire payload bytes, bad messages, payload
 * bytes of launch i.  bank: the uploaded bank (the affixes of the nibble form; NULL: raw payloads) */
int sdx_exchange_count(const sdx_bank* bank, const sdx_xchg_part* parts, int k, void* work_dev, uint64_t work_cap,
                       uint32_t* counts_dev, void* hip_stream);
/* after sdx_exchange_count on the same stream (reads its counts_dev and workspace), the same bank */
int sdx_exchange_pack(const sdx_bank* bank, const sdx_xchg_part* parts, int k, void* work_dev, uint64_t work_cap,
                      const uint32_t* counts_dev, uint8_t* send_dev, uint64_t send_cap, void* hip_stream);
/* ABI 10: the same pack after the counts have reached the host (counts_host = the same u32 counts):
 * dst_dev needs only the exact wire size (16-byte aligned), so the wire can be written straight into
 * this rank's chunk of an in-place all-gather's receive buffer (no send buffer, no local copy) */
int sdx_exchange_pack_into(const sdx_bank* bank, const sdx_xchg_part* parts, int k, void* work_dev, uint64_t work_cap,
                           const uint32_t* counts_dev, const uint32_t* counts_host, uint8_t* dst_dev, uint64_t dst_cap,
                           void* hip_stream);

/* receiver: one launch's wire sections of every rank (rank order = global message order) -> the
 * whole job's sdx_desc[sum n_msgs], sdx_result[sum n_rec] and one contiguous heap (sum n_payload
 * bytes <= heap_cap).  bank / kind: the sender's (the nibble form's affixes).  work_dev:
 * sdx_exchange_unpack_work_bytes(total messages, total records), 64-byte aligned. */
typedef struct {
  const uint8_t* msg_dev;
  const uint8_t* rec_dev;
  const uint8_t* heap_dev;
  uint32_t n_msgs, n_rec, n_heap;  /* n_heap: wire payload bytes (without the padding) */
  uint32_t n_payload;              /* payload bytes they expand to (the count's [4]) */
} sdx_xchg_wire;

uint64_t sdx_exchange_unpack_work_bytes(uint32_t n_msgs, uint32_t n_rec);
int sdx_exchange_unpack(const sdx_bank* bank, int kind, const sdx_xchg_wire* ranks, int nranks, void* work_dev,
                        uint64_t work_cap, sdx_desc* desc_dev, sdx_result* rec_dev, uint8_t* heap_dev,
                        uint64_t heap_cap, void* hip_stream);

#define SDX_SHORT_MAX 256   /* sdx_demod_pulses: messages of <= 256 pulses */
#define SDX_LONG_MAX 4096   /* sdx_demod_pulses_long */
#define SDX_MC_HEX_MAX 128  /* sdx_demod_mc */
#define SDX_MN_HEX_MAX 4096 /* sdx_demod_mn */
/* ABI 14: MC lines of <= SDX_MC_SHORT_HEX characters (SDX_SEL_MC) and longer ones (SDX_SEL_MC_LONG) are
 * separate classes, so a caller knows the short list's length bound (sdx_mc_batch.max_hex, sdx_demod_step) */
enum sdx_sel_class { SDX_SEL_MU_SHORT = 0, SDX_SEL_MU_LONG = 1, SDX_SEL_MS_SHORT = 2, SDX_SEL_MS_LONG = 3,
                     SDX_SEL_MC = 4, SDX_SEL_MC_LONG = 5, SDX_SEL_MN = 6, SDX_SEL_NCLASS = 7 };
#define SDX_SEL_CHUNK 1024  /* lines per selection workgroup */
/* Selection lists for the demodulation launches, built on the device in line order: the OK lines
 * of each class (MS lines whose string gates failed are left out -- they have no results).  Class
 * k's line indices are sel_dev[start_k, start_k + counts[k]) with start_k = counts[0] + ... +
 * counts[k-1]; counts_dev[0..6] receives the class sizes (the only value a host needs back, to size
 * the launches).  scratch_dev: 8 * ceil(n / SDX_SEL_CHUNK) int32.  Pass each list as sel_dev of an
 * sdx_pulse_batch / sdx_mc_batch whose arrays are the sdx_lines_out arrays (offsets = doff_dev,
 * len = dlen_dev, data = slot_dev). */
int sdx_select_lines(const sdx_lines_out* out, int32_t n, int32_t* sel_dev, int32_t* counts_dev,
                     int32_t* scratch_dev, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif
