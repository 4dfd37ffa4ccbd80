// PMC calibration for k_fill's scratch access pattern (diagnostics).
//
// MI355X_MICROARCH.md (HBM): FETCH_SIZE / WRITE_SIZE are calibrated only for
// 16-byte-per-lane streaming accesses; other widths must be calibrated on a
// known byte count.  k_fill's per-wave scratch is written as one dword per
// lane per column (a 256-byte row) plus one byte per lane (a 64-byte row) and
// read back by the traceback one dword (and one byte) per lane-group per
// column.  Each kernel here moves a known number of bytes in exactly those
// shapes over 1 GiB buffers (4x the Infinity Cache, so no line is re-read on
// die), one launch per pattern:
//   0  dword stores, 256 B per wave per row          (k_fill direction words)
//   1  byte stores, 64 B per wave per row            (k_fill match bytes)
//   2  dword loads, 256 B per wave per row           (every lane reads its word)
//   3  dword loads by lane 0 of each 4-lane group, 64 B of each 256-B row
//      (the traceback's per-window reads: one word per group per column)
//   4  16-byte-per-lane stores (the guide's calibrated reference)
//   5  16-byte-per-lane loads (the guide's calibrated reference: FETCH = half)
// usage: pmc_calib [pattern]   (no argument: all six, one launch each)
// Run under rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE; compare with
// the printed byte counts.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static const size_t BYTES = (size_t)1 << 30;
static const int WAVES = 4096;

// each wave owns a contiguous slab of rows of 256 B (dword) or 64 B (byte)
__global__ __launch_bounds__(256) void k_dword_store(uint32_t* p, size_t rows_per_wave, uint32_t v) {
  const size_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  uint32_t* base = p + wave * rows_per_wave * 64;
  for (size_t r = 0; r < rows_per_wave; r++) base[r * 64 + lane] = v + (uint32_t)r;
}
__global__ __launch_bounds__(256) void k_byte_store(uint8_t* p, size_t rows_per_wave, uint32_t v) {
  const size_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  uint8_t* base = p + wave * rows_per_wave * 64;
  for (size_t r = 0; r < rows_per_wave; r++) base[r * 64 + lane] = (uint8_t)(v + r);
}
__global__ __launch_bounds__(256) void k_dword_load(const uint32_t* p, size_t rows_per_wave, uint32_t* out,
                                                    int group_lead_only) {
  const size_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const uint32_t* base = p + wave * rows_per_wave * 64;
  uint32_t acc = 0;
  if (!group_lead_only || (lane & 3) == 0)
    for (size_t r = 0; r < rows_per_wave; r++) acc += base[r * 64 + lane];
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads
}
__global__ __launch_bounds__(256) void k_vec_store(uint4* p, size_t rows_per_wave, uint32_t v) {
  const size_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  uint4* base = p + wave * rows_per_wave * 64;
  for (size_t r = 0; r < rows_per_wave; r++) base[r * 64 + lane] = make_uint4(v, v + 1, v + 2, (uint32_t)r);
}
__global__ __launch_bounds__(256) void k_vec_load(const uint4* p, size_t rows_per_wave, uint32_t* out) {
  const size_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const uint4* base = p + wave * rows_per_wave * 64;
  uint32_t acc = 0;
  for (size_t r = 0; r < rows_per_wave; r++) {
    const uint4 x = base[r * 64 + lane];
    acc += x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  void* buf;
  uint32_t* out;
  CHK(hipMalloc(&buf, BYTES));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(buf, 1, BYTES));
  CHK(hipDeviceSynchronize());
  const dim3 grid(WAVES / 4), block(256);
  const size_t dw_rows = BYTES / 256 / WAVES, b_rows = BYTES / 64 / WAVES, v_rows = BYTES / 1024 / WAVES;
  for (int pat = 0; pat < 6; pat++) {
    if (only >= 0 && pat != only) continue;
    double bytes = 0;
    const char* what = "";
    switch (pat) {
      case 0:
        hipLaunchKernelGGL(k_dword_store, grid, block, 0, 0, (uint32_t*)buf, dw_rows, 7u);
        bytes = (double)WAVES * dw_rows * 256;
        what = "dword stores (256 B rows)";
        break;
      case 1:
        hipLaunchKernelGGL(k_byte_store, grid, block, 0, 0, (uint8_t*)buf, b_rows, 7u);
        bytes = (double)WAVES * b_rows * 64;
        what = "byte stores (64 B rows)";
        break;
      case 2:
        hipLaunchKernelGGL(k_dword_load, grid, block, 0, 0, (const uint32_t*)buf, dw_rows, out, 0);
        bytes = (double)WAVES * dw_rows * 256;
        what = "dword loads, every lane (256 B rows)";
        break;
      case 3:
        hipLaunchKernelGGL(k_dword_load, grid, block, 0, 0, (const uint32_t*)buf, dw_rows, out, 1);
        bytes = (double)WAVES * dw_rows * 64;
        what = "dword loads, one lane in four (64 B of each 256 B row)";
        break;
      case 4:
        hipLaunchKernelGGL(k_vec_store, grid, block, 0, 0, (uint4*)buf, v_rows, 7u);
        bytes = (double)WAVES * v_rows * 1024;
        what = "16 B/lane stores (1 KiB rows)";
        break;
      case 5:
        hipLaunchKernelGGL(k_vec_load, grid, block, 0, 0, (const uint4*)buf, v_rows, out);
        bytes = (double)WAVES * v_rows * 1024;
        what = "16 B/lane loads (1 KiB rows)";
        break;
    }
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    printf("pattern %d: %s: %.0f bytes touched (%.1f KB)\n", pat, what, bytes, bytes / 1024.0);
  }
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return 0;
}
