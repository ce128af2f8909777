// Diagnostic: one-rank RCCL ncclSend/ncclRecv to self, compared byte for byte.
// Round 4 found a 1-rank MG graph build wrong when the alltoallv sent a rank's
// 2.08 GB own share to itself in one ncclSend (RMAT-22's 0.5 GB was exact).  This
// pins the threshold: per size and element type, one send/recv pair of the whole
// buffer, then the same buffer in kPiece-byte pieces (the library's peer path,
// comm.cpp alltoallv), each checked word for word on the device.
//
// build: hipcc -O2 --offload-arch=gfx950 rccl_self.hip -o rccl_self -lrccl
// usage: ./rccl_self [bytes ...]   (defaults: 1.9, 2.0, 2^31-4, 2^31, 2^31+4, 2.2, 4.2 GB)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define NK(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) { printf("RCCL %s line %d\n", ncclGetErrorString(r_), __LINE__); return false; } } while (0)

__device__ __forceinline__ unsigned pattern(size_t i) { return (unsigned)(i * 2654435761ull) ^ (unsigned)(i >> 32) ^ 0x5bd1e995u; }

__global__ void k_fill(unsigned* p, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = pattern(i);
}

// mismatches counted per lane, reduced per block, one vector atomic per block
__global__ void k_check(unsigned const* p, size_t n, unsigned long long* bad, unsigned long long* first)
{
  unsigned long long c = 0, f = ~0ull;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != pattern(i)) {
      ++c;
      if (i < f) f = i;
    }
  if (c) {
    atomicAdd(bad, c);
    atomicMin(first, f);
  }
}

static bool run(ncclComm_t comm, hipStream_t st, size_t bytes, ncclDataType_t dt, size_t es, size_t piece,
                unsigned* src, unsigned* dst, unsigned long long* dctr)
{
  size_t const words = bytes / 4;
  CK(hipMemsetAsync(dst, 0xff, bytes, st));
  size_t const count = bytes / es;
  size_t const pe    = piece ? piece / es : count;
  NK(ncclGroupStart());
  for (size_t o = 0; o < count; o += pe) NK(ncclSend((char*)src + o * es, std::min(pe, count - o), dt, 0, comm, st));
  for (size_t o = 0; o < count; o += pe) NK(ncclRecv((char*)dst + o * es, std::min(pe, count - o), dt, 0, comm, st));
  NK(ncclGroupEnd());
  unsigned long long init[2] = {0, ~0ull};
  CK(hipMemcpyAsync(dctr, init, sizeof(init), hipMemcpyHostToDevice, st));
  k_check<<<4096, 256, 0, st>>>(dst, words, dctr, dctr + 1);
  unsigned long long h[2];
  CK(hipMemcpyAsync(h, dctr, sizeof(h), hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  printf("  %-6s %12zu B (%.3f GB, count %zu, %s): %s", es == 1 ? "uint8" : es == 4 ? "int32" : "int64", bytes,
         bytes / 1e9, pe, piece ? "pieces" : "one send", h[0] ? "MISMATCH" : "exact");
  if (h[0]) printf(" -- %llu bad words, first at byte %llu (%.3f GB)", h[0], h[1] * 4, h[1] * 4 / 1e9);
  printf("\n");
  fflush(stdout);
  return true;
}

int main(int argc, char** argv)
{
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; ++i) sizes.push_back(strtoull(argv[i], nullptr, 10) & ~size_t(7));
  if (sizes.empty())
    sizes = {1900000000ull, 2000000000ull, (1ull << 31) - 8, 1ull << 31, (1ull << 31) + 8, 2200000000ull,
             4200000000ull};
  size_t mx = 0;
  for (size_t s : sizes) mx = s > mx ? s : mx;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return 1;
  ncclComm_t comm;
  if (ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess) return 1;
  unsigned *src, *dst;
  unsigned long long* dctr;
  CK(hipMalloc(&src, mx));
  CK(hipMalloc(&dst, mx));
  CK(hipMalloc(&dctr, 16));
  k_fill<<<4096, 256, 0, st>>>(src, mx / 4);
  CK(hipStreamSynchronize(st));
  printf("one-rank RCCL send/recv to self (RCCL %d)\n", NCCL_VERSION_CODE);
  for (size_t s : sizes) {
    for (auto [dt, es] : {std::pair{ncclInt32, size_t(4)}, std::pair{ncclUint8, size_t(1)}, std::pair{ncclInt64, size_t(8)}})
      if (!run(comm, st, s, dt, es, 0, src, dst, dctr)) return 1;
    if (!run(comm, st, s, ncclInt32, 4, size_t(1) << 30, src, dst, dctr)) return 1;
  }
  ncclCommDestroy(comm);
  return 0;
}
