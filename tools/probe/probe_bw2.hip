// Dev probe (not product): streaming-write rate on one MI355X by store width, grid size, workgroup
// size and cache policy, for the soft-assign's 6.4 GB responsibility stream (which writes dwordx4
// non-temporal rows at ~4.9 TB/s, profiles/r05/probe_bw_session1.txt). Each kernel writes the whole
// buffer once with a grid-stride loop; rate = bytes / time of the second of two launches.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int W, int POL>  // W: bytes per lane per store (4, 8, 16); POL 0 plain, 1 nt
__global__ void k_w(char* __restrict__ out, long bytes) {
  const long n = bytes / W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if constexpr (W == 16) {
      d2 v = d2{1.0, 2.0};
      if (POL) __builtin_nontemporal_store(v, reinterpret_cast<d2*>(out) + i);
      else reinterpret_cast<d2*>(out)[i] = v;
    } else if constexpr (W == 8) {
      if (POL) __builtin_nontemporal_store(1.0, reinterpret_cast<double*>(out) + i);
      else reinterpret_cast<double*>(out)[i] = 1.0;
    } else {
      if (POL) __builtin_nontemporal_store(1.0f, reinterpret_cast<float*>(out) + i);
      else reinterpret_cast<float*>(out)[i] = 1.0f;
    }
  }
}
// each wave writes whole 4 KiB pages in turn (16 B per lane, 4 instructions per page): a page per wave
template <int POL>
__global__ void k_wpage(char* __restrict__ out, long bytes) {
  const long pages = bytes / 4096;
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long p = wave; p < pages; p += nw) {
    d2* base = reinterpret_cast<d2*>(out + p * 4096);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d2 v = d2{1.0, 2.0};
      if (POL) __builtin_nontemporal_store(v, base + k * 64 + lane);
      else base[k * 64 + lane] = v;
    }
  }
}

template <typename K>
static void run(const char* name, K kern, int grid, int block, char* buf, long bytes) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0.f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, buf, bytes);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  printf("%-10s grid %6d block %4d  %.2f TB/s\n", name, grid, block, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

int main() {
  const long bytes = 6400L << 20;
  char* buf;
  if (hipMalloc(&buf, bytes)) return 1;
  for (int block : {256, 512, 1024})
    for (int grid : {512, 1024, 2048, 8192, 32768}) {
      run("w16", k_w<16, 0>, grid, block, buf, bytes);
      run("w16nt", k_w<16, 1>, grid, block, buf, bytes);
      run("w8", k_w<8, 0>, grid, block, buf, bytes);
      run("w8nt", k_w<8, 1>, grid, block, buf, bytes);
      run("w4", k_w<4, 0>, grid, block, buf, bytes);
      run("page", k_wpage<0>, grid, block, buf, bytes);
      run("pagent", k_wpage<1>, grid, block, buf, bytes);
    }
  return 0;
}
