// Measurement tool (not product): what one 4-byte gather instruction costs a CU's
// vector-memory path (TA / TCP / TD) as a function of how many distinct 128-B lines
// its 64 lanes touch and how many lanes are active -- the question behind the
// PageRank push's "cached floor" (profiles/r03_push_pmc.md: TA 71 % / TD 80 % busy,
// ~28 TA cycles per VMEM instruction with every x~ line cached).
//
//   gather_cost <table_KB> <lines> <active_lanes> [iters]
//     lines = 0: every lane reads the same dword; L >= 1: lane l reads dword l % 32 of
//     line (l * L / 64) of the instruction's L consecutive lines (L <= 64); the lines
//     move on every instruction and wrap inside the table, so a small table stays in
//     the L1 / L2 and only the per-instruction cost is left.
//
// Prints: table KB, lines, lanes, ms, cycles per gather instruction per CU (2.4 GHz,
// 256 CUs, wave instructions spread evenly).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench/gather_cost scripts/ubench/gather_cost.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int kU = 8;  // independent gathers in flight per lane

__global__ __launch_bounds__(256) void k_gcost(float const* __restrict__ table, unsigned mask_lines, int lines,
                                               int active, int iters, float* out)
{
  int const lane     = threadIdx.x & 63;
  unsigned const wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  unsigned line0     = (wid * 977u) & mask_lines;
  unsigned const sub = lines ? (unsigned)(lane * lines / 64) : 0u;
  unsigned const off = lines ? (unsigned)(lane & 31) : 0u;
  unsigned const step = lines ? (unsigned)lines : 1u;
  float acc[kU] = {};
  bool const on = lane < active;
  for (int it = 0; it < iters; it += kU) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      unsigned const l = (line0 + (unsigned)(it + u) * step + sub) & mask_lines;
      if (on) acc[u] += table[l * 32u + off];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < kU; ++u) s += acc[u];
  if (s == 12345.f) out[0] = s;  // keeps the loads
}

int main(int argc, char** argv)
{
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <table_KB> <lines> <active_lanes> [iters]\n", argv[0]);
    return 2;
  }
  long const kb    = std::atol(argv[1]);
  int const lines  = std::atoi(argv[2]);
  int const active = std::atoi(argv[3]);
  int const iters  = argc > 4 ? std::atoi(argv[4]) : 2048;
  long const nlines = kb * 1024 / 128;
  if (nlines < 64 || (nlines & (nlines - 1)) || lines < 0 || lines > 64 || active < 1 || active > 64 ||
      iters % kU) {
    std::fprintf(stderr, "table must be a power of two >= 8 KB, 0 <= lines <= 64, 1 <= lanes <= 64\n");
    return 2;
  }
  float* table;
  float* out;
  CK(hipMalloc(&table, nlines * 128));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(table, 0, nlines * 128));
  int const grid = 2048, block = 256;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ms;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_gcost, dim3(grid), dim3(block), 0, 0, table, (unsigned)(nlines - 1), lines, active, iters,
                       out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float t;
    CK(hipEventElapsedTime(&t, a, b));
    if (r) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  double const t      = ms[ms.size() / 2];
  double const instrs = (double)grid * (block / 64) * iters / 256.0;  // per CU
  std::printf("table_KB %ld lines %d lanes %d ms %.4f cycles/instr/CU %.2f\n", kb, lines, active, t,
              t * 1e-3 * 2.4e9 / instrs);
  CK(hipFree(table));
  CK(hipFree(out));
  return 0;
}
