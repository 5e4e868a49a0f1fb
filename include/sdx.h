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

#define SDX_ABI_VERSION 1

enum { SDX_OK = 0, SDX_EINVAL = -1, SDX_EHIP = -2, SDX_EBANK = -3, SDX_ECONTRACT = -4 };

enum sdx_kind { SDX_KIND_MU = 0, SDX_KIND_MS = 1, SDX_KIND_MC = 2 };

/* per-message status in sdx_desc.status */
enum sdx_status {
  SDX_ST_OK = 0,       /* results [rec_begin, rec_begin+n_rec) are the reference's list */
  SDX_ST_RAISED = 1,   /* the reference raises: raise_kind says which exception */
  SDX_ST_OVF_TILE = 2, /* on-chip result staging overflowed: re-run this message */
  SDX_ST_OVF_OUT = 3   /* the caller's result/heap capacity overflowed: grow and re-run */
};
/* sdx_desc.raise_kind (Python exception class the reference raises) */
enum sdx_raise { SDX_RAISE_NONE = 0, SDX_RAISE_INDEX = 1, SDX_RAISE_ATTRIBUTE = 2, SDX_RAISE_VALUE = 3,
                 SDX_RAISE_TYPE = 4, SDX_RAISE_ZERODIV = 5 };

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

/* MU / MS batch: structure-of-arrays in HBM (see DESIGN.md "Data layout") */
typedef struct {
  const uint8_t* data_dev;     /* pulse-id characters, all messages concatenated */
  const int64_t* offsets_dev;  /* [n+1] message i = data[offsets[i], offsets[i+1]) */
  const uint8_t* npat_dev;     /* [n] number of P# patterns (<= 10) */
  const uint8_t* pat_id_dev;   /* [n*10] ASCII id digit of pattern slot k, dict order */
  const double* pat_val_dev;   /* [n*10] float(P#) */
  const int8_t* cp_slot_dev;   /* [n] MS: slot of CP, -1 = CP not a pattern (NULL for MU) */
  const uint8_t* ms_ok_dev;    /* [n] MS: CP/SP/R string gates passed (NULL for MU) */
  const int32_t* sel_dev;      /* optional [n_sel] subset of message indices to run, NULL = all */
  int32_t n;                   /* messages in the batch */
  int32_t n_sel;               /* entries in sel_dev (ignored when sel_dev == NULL) */
} sdx_pulse_batch;

/* MC batch */
typedef struct {
  const uint8_t* hex_dev;      /* hex characters (D=) of all frames concatenated */
  const int64_t* offsets_dev;  /* [n+1] */
  const int32_t* clock_dev;    /* [n] C= */
  const int32_t* mcbitnum_dev; /* [n] L= */
  const uint8_t* flags_dev;    /* [n] bit0: message type 'Mc', bit1: version starts 'V 3.2.' */
  const int32_t* sel_dev;
  int32_t n, n_sel;
} sdx_mc_batch;

/* output buffers (caller-owned, device) */
typedef struct {
  sdx_desc* desc_dev;          /* [n] */
  sdx_result* rec_dev;         /* [rec_cap] */
  uint8_t* heap_dev;           /* [heap_cap] */
  uint32_t* cursor_dev;        /* [4] zeroed by the caller before the first launch: rec, heap, ovf */
  uint32_t rec_cap, heap_cap;
} sdx_out;

typedef struct sdx_bank sdx_bank;

int sdx_abi_version(void);
const char* sdx_last_error(void);
/* sizeof() of the bank records, for host layout checks: 0 hdr, 1 patspec, 2 mu, 3 ms, 4 mc, 5 result, 6 desc,
 * 7 mu_desc */
int sdx_layout_size(int which);

/* bank: compiled by pysignalduino_amd/bank.py (protocols.json -> blob) and uploaded once per device */
int sdx_bank_create(const void* blob, size_t nbytes, int device, sdx_bank** out);
int sdx_bank_destroy(sdx_bank* bank);
const void* sdx_bank_device_ptr(const sdx_bank* bank);

/* MU/MS demodulation of a batch: one launch, results appended to out */
int sdx_demod_pulses(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, const sdx_out* out,
                     void* hip_stream);
/* same, for messages of 257..4096 pulses (4 messages per workgroup tile) */
int sdx_demod_pulses_long(const sdx_bank* bank, int kind, const sdx_pulse_batch* batch, const sdx_out* out,
                          void* hip_stream);
/* MC "fixed" chain: every frame x every clockrange protocol */
int sdx_demod_mc(const sdx_bank* bank, const sdx_mc_batch* batch, const sdx_out* out, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif
