// sdx_exchange.hip -- the device side of the multi-GPU exchange (BASELINE config 5).
//
// Every rank demodulates its contiguous shard of the stream; the one exchange step all-gathers the
// decoded dmsg buffers (descriptors, result records, payload heap) of all ranks over RCCL.  Before
// the all-gather, each rank packs its buffers of K launches (MU, MS, MC) into one send buffer and
// re-bases them to the whole job's numbering while copying: rec_begin += records of the lower
// ranks, payload_off += heap bytes of the lower ranks, msg += messages of the lower ranks.  One
// launch does all K launches' sections (blockIdx.y = section), 16-byte vector copies for the heap,
// one thread per descriptor / record for the re-based sections.  No host round trip: the host only
// passes the counts it already read for sizing the collective.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/sdx.h"

namespace sdx {
int set_error(int code, const std::string& msg);  // sdx_kernels.hip
}

namespace sdxx {

constexpr int XT = 256;
constexpr int XMAX = 8;  // launches per exchange

struct Parts {
  sdx_xchg_part p[XMAX];
};

__global__ __launch_bounds__(XT) void k_exchange_pack(Parts P, uint8_t* __restrict__ send) {
  const int s = blockIdx.y, part = s / 3, sec = s % 3;
  const sdx_xchg_part& x = P.p[part];
  const size_t stride = (size_t)gridDim.x * XT;
  const size_t t0 = (size_t)blockIdx.x * XT + threadIdx.x;
  if (sec == 0) {  // descriptors: rec_begin re-based
    const sdx_desc* d = reinterpret_cast<const sdx_desc*>(x.desc_dev);
    sdx_desc* o = reinterpret_cast<sdx_desc*>(send + x.off_desc);
    for (size_t i = t0; i < x.n_msgs; i += stride) {
      sdx_desc v = d[i];
      v.rec_begin += x.base_rec;
      o[i] = v;
    }
  } else if (sec == 1) {  // records: payload_off and msg re-based
    const sdx_result* r = reinterpret_cast<const sdx_result*>(x.rec_dev);
    sdx_result* o = reinterpret_cast<sdx_result*>(send + x.off_rec);
    for (size_t i = t0; i < x.n_rec; i += stride) {
      sdx_result v = r[i];
      v.payload_off += x.base_heap;
      v.msg += x.base_msg;
      o[i] = v;
    }
  } else {  // heap: 16-byte pieces (heap and section offsets are 16-byte aligned), then the tail
    const uint4* h = reinterpret_cast<const uint4*>(x.heap_dev);
    uint4* o = reinterpret_cast<uint4*>(send + x.off_heap);
    const size_t nv = x.n_heap / 16;
    for (size_t i = t0; i < nv; i += stride) o[i] = h[i];
    for (size_t i = nv * 16 + t0; i < x.n_heap; i += stride) send[x.off_heap + i] = x.heap_dev[i];
  }
}

}  // namespace sdxx

extern "C" int sdx_exchange_pack(const sdx_xchg_part* parts, int k, uint8_t* send_dev, void* hip_stream) {
  if (!parts || !send_dev || k < 1 || k > sdxx::XMAX) return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack: bad arguments");
  sdxx::Parts P;
  size_t most = 1;
  for (int i = 0; i < sdxx::XMAX; ++i) P.p[i] = i < k ? parts[i] : sdx_xchg_part{};
  for (int i = 0; i < k; ++i) {
    const sdx_xchg_part& x = parts[i];
    if ((x.off_desc & 7u) || (x.off_rec & 15u) || (x.off_heap & 15u) || (((uintptr_t)x.heap_dev) & 15u) ||
        (((uintptr_t)send_dev) & 15u))
      return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack: sections and heap must be 16-byte aligned");
    if ((x.n_msgs && !x.desc_dev) || (x.n_rec && !x.rec_dev) || (x.n_heap && !x.heap_dev))
      return sdx::set_error(SDX_EINVAL, "sdx_exchange_pack: missing buffer");
    most = x.n_msgs > most ? x.n_msgs : most;
    most = x.n_rec > most ? x.n_rec : most;
    most = x.n_heap / 16 > most ? x.n_heap / 16 : most;
  }
  size_t blocks = (most + sdxx::XT - 1) / sdxx::XT;
  if (blocks > 2048) blocks = 2048;  // grid-stride beyond: >= 8 blocks per CU already
  hipLaunchKernelGGL(sdxx::k_exchange_pack, dim3((unsigned)blocks, 3 * k), dim3(sdxx::XT), 0, (hipStream_t)hip_stream,
                     P, send_dev);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sdx::set_error(SDX_EHIP, std::string("k_exchange_pack: ") + hipGetErrorString(e));
  return SDX_OK;
}
