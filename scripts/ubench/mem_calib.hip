// Measurement tool (not product): calibrates what the rocprofv3 HBM counters mean for
// the two access shapes of the PageRank push, and finds the copy ceiling.
//
//   copy  <MB> <block> <unroll> <grid> <nt>   16-B-per-lane grid-stride copy (read + write)
//   read  <MB> <block> <unroll> <grid>        16-B-per-lane streaming read (sum)
//   gather <table_MB> <n_millions> <grid>     random 4-B gathers from a table, addresses
//                                             from a hash (no index stream): every gather
//                                             touches a line no other gather of the launch
//                                             is likely to share when the table is large
//   gatherk <table_MB> <n_millions> <grid> <aux>  the same through raw buffer loads with
//                                             cache-policy bits aux (gfx940+: 1 sc0, 2 nt,
//                                             16 sc1): which policy fills a 4-B miss with
//                                             fewer fabric bytes (TCC_EA0_RDREQ_32B_sum)
//   streamgather <table_MB> <stream_MB> <grid> <aux>  per lane: one 16-B load of a stream
//                                             read once (cache policy aux) and 4 random
//                                             4-B gathers from a small table (plain): does
//                                             the stream's policy keep the table in L2?
//                                             (the push's entry stream beside its x~ gathers)
//
// Prints one line per run: mode, bytes the kernel asks for, ms per launch (HIP events,
// median of reps), GB/s or Ggathers/s.  Under `rocprofv3 --pmc FETCH_SIZE` (or
// TCC_EA0_RDREQ_sum etc.) the counter per launch divided by the known request count
// gives the bytes one request is tallied at for that shape.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench/mem_calib scripts/ubench/mem_calib.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void k_copy(u32x4 const* __restrict__ src, u32x4* __restrict__ dst, long n)
{
  long const stride = (long)gridDim.x * blockDim.x;
  long i            = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = NT ? __builtin_nontemporal_load(src + i + j * stride) : src[i + j * stride];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (NT) __builtin_nontemporal_store(v[j], dst + i + j * stride);
      else dst[i + j * stride] = v[j];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

template <int U>
__global__ void k_read(u32x4 const* __restrict__ src, long n, unsigned* out)
{
  long const stride = (long)gridDim.x * blockDim.x;
  long i            = blockIdx.x * (long)blockDim.x + threadIdx.x;
  unsigned acc      = 0;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = __builtin_nontemporal_load(src + i + j * stride);
#pragma unroll
    for (int j = 0; j < U; ++j) acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  for (; i < n; i += stride) acc += src[i].x;
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads live
}

__device__ inline unsigned mix(unsigned long long x)
{
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (unsigned)x;
}

// 8 independent gathers per lane per round; addresses are hashes of the global
// gather number, so every launch reads the same multiset of words
__global__ void k_gather(float const* __restrict__ table, unsigned nwords, long ngather, float* out)
{
  long const stride = (long)gridDim.x * blockDim.x * 8;
  float acc         = 0.f;
  for (long b = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 8; b < ngather; b += stride) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = table[mix((unsigned long long)(b + j)) % nwords];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  if (acc == 1234.5f) out[0] = acc;
}

template <int AUX>
__global__ void k_gather_aux(float const* __restrict__ table, unsigned nwords, long ngather, float* out)
{
  __amdgpu_buffer_rsrc_t const r =
    __builtin_amdgcn_make_buffer_rsrc((void*)table, (short)0, (int)(nwords * 4u), 0x00020000);
  long const stride = (long)gridDim.x * blockDim.x * 8;
  float acc         = 0.f;
  for (long b = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 8; b < ngather; b += stride) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (mix((unsigned long long)(b + j)) % nwords) * 4u, 0, AUX));
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  if (acc == 1234.5f) out[0] = acc;
}

template <int AUX>
__global__ void k_stream_gather(u32x4 const* __restrict__ stream, long n16, float const* __restrict__ table,
                                unsigned nwords, float* out)
{
  __amdgpu_buffer_rsrc_t const r = __builtin_amdgcn_make_buffer_rsrc((void*)stream, (short)0, 0x7fffffff, 0x00020000);
  long const stride = (long)gridDim.x * blockDim.x;
  unsigned acc      = 0;
  float facc        = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += stride) {
    // offsets within the first 2 GB of the stream (n16 * 16 < 2^31)
    u32x4 const v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(i * 16), 0, AUX));
    float g[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = table[mix((unsigned long long)(i * 4 + j)) % nwords];
    acc += v.x ^ v.w;
#pragma unroll
    for (int j = 0; j < 4; ++j) facc += g[j];
  }
  if (acc == 0x9e3779b9u || facc == 1234.5f) out[0] = facc;
}

template <typename F>
static float time_ms(F&& launch, int reps)
{
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv)
{
  if (argc < 2) {
    std::fprintf(stderr, "usage: see the header\n");
    return 2;
  }
  int const reps = std::getenv("REPS") ? std::atoi(std::getenv("REPS")) : 10;
  std::string const mode = argv[1];
  if (mode == "copy" || mode == "read") {
    size_t const mb  = std::strtoull(argv[2], nullptr, 10);
    int const block  = std::atoi(argv[3]);
    int const unroll = std::atoi(argv[4]);
    int const grid   = std::atoi(argv[5]);
    bool const nt    = argc > 6 ? std::atoi(argv[6]) != 0 : true;
    long const n     = (long)(mb << 20) / 16;
    u32x4 *a, *b;
    unsigned* out;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(a, 1, n * 16));
    CK(hipMemset(b, 2, n * 16));
    auto launch = [&]() {
      if (mode == "read") {
        switch (unroll) {
          case 4: hipLaunchKernelGGL(k_read<4>, dim3(grid), dim3(block), 0, 0, a, n, out); break;
          case 8: hipLaunchKernelGGL(k_read<8>, dim3(grid), dim3(block), 0, 0, a, n, out); break;
          default: hipLaunchKernelGGL(k_read<16>, dim3(grid), dim3(block), 0, 0, a, n, out); break;
        }
        return;
      }
#define CASE(U)                                                                                   \
  case U:                                                                                         \
    if (nt) hipLaunchKernelGGL((k_copy<U, true>), dim3(grid), dim3(block), 0, 0, a, b, n);        \
    else hipLaunchKernelGGL((k_copy<U, false>), dim3(grid), dim3(block), 0, 0, a, b, n);          \
    break;
      switch (unroll) {
        CASE(1)
        CASE(2)
        CASE(4)
        CASE(8)
        default: CASE(16)
      }
#undef CASE
    };
    float const ms    = time_ms(launch, reps);
    double const byts = (mode == "copy" ? 2.0 : 1.0) * n * 16;
    std::printf("%s MB=%zu block=%d unroll=%d grid=%d nt=%d bytes=%.0f ms=%.4f GB/s=%.1f\n", mode.c_str(), mb, block,
                unroll, grid, (int)nt, byts, ms, byts / (ms * 1e-3) / 1e9);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(out));
  } else if (mode == "gather") {
    size_t const mb  = std::strtoull(argv[2], nullptr, 10);
    long const ng    = (long)(std::atof(argv[3]) * 1e6);
    int const grid   = argc > 4 ? std::atoi(argv[4]) : 4096;
    unsigned const nw = (unsigned)((mb << 20) / 4);
    float* t;
    float* out;
    CK(hipMalloc(&t, (size_t)nw * 4));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(t, 0, (size_t)nw * 4));
    auto launch = [&]() { hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, 0, t, nw, ng, out); };
    float const ms = time_ms(launch, reps);
    std::printf("gather table_MB=%zu gathers=%ld grid=%d ms=%.4f Ggather/s=%.2f GB/s@128B=%.1f GB/s@64B=%.1f "
                "GB/s@32B=%.1f\n",
                mb, ng, grid, ms, ng / (ms * 1e-3) / 1e9, 128.0 * ng / (ms * 1e-3) / 1e9,
                64.0 * ng / (ms * 1e-3) / 1e9, 32.0 * ng / (ms * 1e-3) / 1e9);
    CK(hipFree(t));
    CK(hipFree(out));
  } else if (mode == "gatherk") {
    size_t const mb  = std::strtoull(argv[2], nullptr, 10);
    long const ng    = (long)(std::atof(argv[3]) * 1e6);
    int const grid   = std::atoi(argv[4]);
    int const aux    = std::atoi(argv[5]);
    unsigned const nw = (unsigned)((mb << 20) / 4);
    float* t;
    float* out;
    CK(hipMalloc(&t, (size_t)nw * 4));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(t, 0, (size_t)nw * 4));
    auto launch = [&]() {
      switch (aux) {
#define CASE(A) case A: hipLaunchKernelGGL(k_gather_aux<A>, dim3(grid), dim3(256), 0, 0, t, nw, ng, out); break;
        CASE(0) CASE(1) CASE(2) CASE(3) CASE(16) CASE(17) CASE(18) CASE(19)
#undef CASE
        default: std::fprintf(stderr, "aux must be 0,1,2,3,16,17,18,19\n"); std::exit(2);
      }
    };
    float const ms = time_ms(launch, reps);
    std::printf("gatherk aux=%d table_MB=%zu gathers=%ld grid=%d ms=%.4f Ggather/s=%.2f\n", aux, mb, ng, grid, ms,
                ng / (ms * 1e-3) / 1e9);
    CK(hipFree(t));
    CK(hipFree(out));
  } else if (mode == "streamgather") {
    size_t const tmb = std::strtoull(argv[2], nullptr, 10);
    size_t const smb = std::strtoull(argv[3], nullptr, 10);
    int const grid   = std::atoi(argv[4]);
    int const aux    = std::atoi(argv[5]);
    unsigned const nw = (unsigned)((tmb << 20) / 4);
    long const n16    = (long)(smb << 20) / 16;
    float *t, *out;
    u32x4* st;
    CK(hipMalloc(&t, (size_t)nw * 4));
    CK(hipMalloc(&st, (size_t)n16 * 16));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(t, 0, (size_t)nw * 4));
    CK(hipMemset(st, 1, (size_t)n16 * 16));
    auto launch = [&]() {
      switch (aux) {
#define CASE(A) case A: hipLaunchKernelGGL(k_stream_gather<A>, dim3(grid), dim3(256), 0, 0, st, n16, t, nw, out); break;
        CASE(0) CASE(1) CASE(2) CASE(3) CASE(16) CASE(17) CASE(18) CASE(19)
#undef CASE
        default: std::fprintf(stderr, "aux must be 0,1,2,3,16,17,18,19\n"); std::exit(2);
      }
    };
    float const ms = time_ms(launch, reps);
    std::printf("streamgather aux=%d table_MB=%zu stream_MB=%zu grid=%d ms=%.4f stream GB/s=%.1f Ggather/s=%.2f\n",
                aux, tmb, smb, grid, ms, n16 * 16.0 / (ms * 1e-3) / 1e9, n16 * 4.0 / (ms * 1e-3) / 1e9);
    CK(hipFree(t));
    CK(hipFree(st));
    CK(hipFree(out));
  } else {
    std::fprintf(stderr, "unknown mode\n");
    return 2;
  }
  return 0;
}
