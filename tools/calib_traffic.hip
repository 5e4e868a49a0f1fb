// calib_traffic.hip -- calibration of the rocprofv3 HBM counters (FETCH_SIZE / WRITE_SIZE) on gfx950
// for the access widths this build's kernels use.  MI355X_MICROARCH.md (HBM section)
// states FETCH_SIZE = exactly half the bytes of a wide coalesced 16-B/lane streaming read and leaves
// every other width uncalibrated; k_pulses<MU> reads mostly bytes, dwords, gathered 8-B fields and
// scalar bank records.  Each kernel below moves a KNOWN number of bytes with one access pattern; the
// host prints those byte counts, and tools/calib_traffic.sh runs the binary under separate
// `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes; tools/calib_traffic.py joins the two into
// counter / known-bytes ratios per pattern (profiles/r05/calib_traffic.json).
//
// Buffers are 512 MiB (twice the Infinity Cache) and each pattern touches every byte once, in a
// launch of its own; stores are plain vector stores.
//   usage: ./calib_traffic            (prints one "name bytes_read bytes_written" line per kernel)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

constexpr size_t BUF = 512ull << 20;

// one dword per block keeps the loads alive (negligible writes: grid * 4 bytes)
__device__ void sink(uint32_t* out, uint32_t acc) {
  __shared__ uint32_t s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicXor(&s, acc);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// 16 B per lane, coalesced (the guide's calibrated case)
__global__ void k_rd16(const uint4* __restrict__ a, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  sink(out, acc);
}
// 4 B per lane, coalesced
__global__ void k_rd4(const uint32_t* __restrict__ a, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    acc ^= a[i];
  sink(out, acc);
}
// 1 B per lane, coalesced
__global__ void k_rd1(const uint8_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += a[i];
  sink(out, acc);
}
// one 8-B load per 128-B line, lines in a permuted order (a gathered per-message field): known bytes
// = 8 per line; the line is 128 B
__global__ void k_gather8(const uint64_t* __restrict__ a, const uint32_t* __restrict__ perm, size_t nlines,
                          uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t v = a[(size_t)perm[i] * 16];
    acc ^= (uint32_t)v ^ (uint32_t)(v >> 32);
  }
  sink(out, acc);
}
// wave-uniform (scalar) loads: each wave reads its 256-B chunks with a uniform address
__global__ void k_scalar(const uint32_t* __restrict__ a, size_t nchunks, uint32_t* out) {
  uint32_t acc = 0;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t c = wave; c < nchunks; c += nwaves) {
    const uint32_t* p = a + __builtin_amdgcn_readfirstlane((uint32_t)c) * (size_t)64;
#pragma unroll
    for (int k = 0; k < 64; k += 8) {
      uint32_t x = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) x ^= p[k + j];
      acc ^= x;
    }
  }
  sink(out, acc);
}
// k_pulses<MU>'s global read mix, per 64-message tile in a permuted (grouped) message order: the
// message's 8-B offset, its 1-B npat, its 10 1-B pattern ids and 10 8-B pattern values (one thread per
// (message, pattern)), and its 256 characters as five dword loads per lane at a 16-B lane stride
// (16 lanes per message), exactly as k_pulses stages them.  SoA arrays like sdx_pulse_batch.
struct MuSoA {
  const int64_t* off;
  const uint8_t* npat;
  const uint8_t* pid;
  const double* pval;
  const uint8_t* data;
  const int32_t* sel;
  int n;
};
__global__ __launch_bounds__(512) void k_mu_mix(MuSoA b, uint32_t* out) {
  const int tile0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t acc = 0;
  __shared__ int msg_of[64];
  if (tid < 64) msg_of[tid] = tile0 + tid < b.n ? b.sel[tile0 + tid] : 0;
  __syncthreads();
  for (int i = tid; i < 640; i += 512) {  // (message, pattern) threads
    const int m = i / 10, k = i % 10;
    if (tile0 + m < b.n) {
      const int msg = msg_of[m];
      acc += b.npat[msg] + b.pid[msg * 10 + k];
      const double v = b.pval[msg * 10 + k];
      acc ^= (uint32_t)__double_as_longlong(v);
    }
  }
  for (int ps = 0; ps < 2; ++ps) {  // wave w: tile messages w + 8 k, 4 per pass
    const int k = ps * 4 + (lane >> 4);
    const int mi = wave + 8 * k;
    if (tile0 + mi < b.n) {
      const int msg = msg_of[mi];
      const int64_t base = b.off[msg] + 16 * (lane & 15);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(b.data + (base & ~(int64_t)3));
#pragma unroll
      for (int j = 0; j < 5; ++j) acc ^= (((base & ~3) + 4 * j) < b.off[msg] + 256) ? src[j] : 0u;
    }
  }
  sink(out, acc);
}
// stores: 16 B per lane coalesced, 1 B per lane coalesced, one 8-B store per 128-B line permuted
// (the scattered descriptor / wire-count stores of the k_pulses flush)
__global__ void k_wr16(uint4* __restrict__ a, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ void k_wr1(uint8_t* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (uint8_t)i;
}
__global__ void k_scatter8(uint64_t* __restrict__ a, const uint32_t* __restrict__ perm, size_t nlines) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x)
    a[(size_t)perm[i] * 16] = i;
}
// 8-B stores at consecutive 8-B slots of a permuted message order (descriptor array of n messages,
// every slot written once: the known bytes ARE the array)
__global__ void k_scatter8_dense(uint64_t* __restrict__ a, const uint32_t* __restrict__ perm, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[perm[i]] = i;
}

int main() {
  uint8_t *A, *W;
  uint32_t *out, *perm, *perm_d;
  CHK(hipMalloc(&A, BUF));
  CHK(hipMalloc(&W, BUF));
  CHK(hipMalloc(&out, 1 << 20));
  CHK(hipMemset(A, 0x5A, BUF));
  const size_t nlines = BUF / 128;
  const size_t ndense = BUF / 8 / 8;  // a 64 MiB descriptor array
  std::vector<uint32_t> h(nlines > ndense ? nlines : ndense);
  uint64_t s = 88172645463325252ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (size_t i = 0; i < nlines; ++i) h[i] = (uint32_t)i;
  for (size_t i = nlines - 1; i > 0; --i) std::swap(h[i], h[rnd() % (i + 1)]);
  CHK(hipMalloc(&perm, nlines * 4));
  CHK(hipMemcpy(perm, h.data(), nlines * 4, hipMemcpyHostToDevice));
  for (size_t i = 0; i < ndense; ++i) h[i] = (uint32_t)i;
  for (size_t i = ndense - 1; i > 0; --i) std::swap(h[i], h[rnd() % (i + 1)]);
  CHK(hipMalloc(&perm_d, ndense * 4));
  CHK(hipMemcpy(perm_d, h.data(), ndense * 4, hipMemcpyHostToDevice));
  // the MU mix: n messages of 256 characters, SoA fields, a random permutation as the grouped order
  const int nmsg = 1 << 20;
  int64_t* off;
  uint8_t *npat, *pid, *data;
  double* pval;
  int32_t* sel;
  CHK(hipMalloc(&off, (nmsg + 1) * 8));
  CHK(hipMalloc(&npat, nmsg));
  CHK(hipMalloc(&pid, nmsg * 10));
  CHK(hipMalloc(&pval, nmsg * 80));
  CHK(hipMalloc(&data, (size_t)nmsg * 256 + 64));
  CHK(hipMalloc(&sel, nmsg * 4));
  {
    std::vector<int64_t> ho(nmsg + 1);
    for (int i = 0; i <= nmsg; ++i) ho[i] = (int64_t)i * 256;
    CHK(hipMemcpy(off, ho.data(), ho.size() * 8, hipMemcpyHostToDevice));
    std::vector<int32_t> hs(nmsg);
    for (int i = 0; i < nmsg; ++i) hs[i] = i;
    for (int i = nmsg - 1; i > 0; --i) std::swap(hs[i], hs[rnd() % (i + 1)]);
    CHK(hipMemcpy(sel, hs.data(), nmsg * 4, hipMemcpyHostToDevice));
    CHK(hipMemset(npat, 8, nmsg));
    CHK(hipMemset(pid, '3', nmsg * 10));
    CHK(hipMemset(pval, 0, nmsg * 80));
    CHK(hipMemset(data, '1', (size_t)nmsg * 256 + 64));
  }
  const int grid = 256 * 16, bs = 256;
  auto run = [&](const char* name, size_t rd, size_t wr, auto launch) {
    launch();
    CHK(hipDeviceSynchronize());
    std::printf("%s %zu %zu\n", name, rd, wr);
  };
  run("k_rd16", BUF, 0, [&] { hipLaunchKernelGGL(k_rd16, dim3(grid), dim3(bs), 0, 0, (const uint4*)A, BUF / 16, out); });
  run("k_rd4", BUF, 0, [&] { hipLaunchKernelGGL(k_rd4, dim3(grid), dim3(bs), 0, 0, (const uint32_t*)A, BUF / 4, out); });
  run("k_rd1", BUF, 0, [&] { hipLaunchKernelGGL(k_rd1, dim3(grid), dim3(bs), 0, 0, A, BUF, out); });
  run("k_gather8", nlines * 8, 0,
      [&] { hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(bs), 0, 0, (const uint64_t*)A, perm, nlines, out); });
  run("k_scalar", BUF, 0,
      [&] { hipLaunchKernelGGL(k_scalar, dim3(grid), dim3(bs), 0, 0, (const uint32_t*)A, BUF / 256, out); });
  // known bytes of the MU mix: per message 8 (offset) + 1 (npat) + 10 (ids) + 80 (values) + 256 (data)
  // + 4 (sel); the sel array is read coalesced
  MuSoA mb{off, npat, pid, pval, data, sel, nmsg};
  run("k_mu_mix", (size_t)nmsg * (8 + 1 + 10 + 80 + 256 + 4), 0,
      [&] { hipLaunchKernelGGL(k_mu_mix, dim3(nmsg / 64), dim3(512), 0, 0, mb, out); });
  run("k_wr16", 0, BUF, [&] { hipLaunchKernelGGL(k_wr16, dim3(grid), dim3(bs), 0, 0, (uint4*)W, BUF / 16); });
  run("k_wr1", 0, BUF, [&] { hipLaunchKernelGGL(k_wr1, dim3(grid), dim3(bs), 0, 0, W, BUF); });
  run("k_scatter8", 0, nlines * 8,
      [&] { hipLaunchKernelGGL(k_scatter8, dim3(grid), dim3(bs), 0, 0, (uint64_t*)W, perm, nlines); });
  run("k_scatter8_dense", 0, ndense * 8,
      [&] { hipLaunchKernelGGL(k_scatter8_dense, dim3(grid), dim3(bs), 0, 0, (uint64_t*)W, perm_d, ndense); });
  CHK(hipFree(A));
  CHK(hipFree(W));
  return 0;
}
