// Microbenchmark: cycles per dependent float64 op for ONE wave alone on a
// SIMD, with 1, 2 and 4 independent chains, and per sqrt/div/sincos.
// Shader-clock (s_memtime) stamps; one workgroup of 64 threads (or W waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

template <int C>
__global__ void chain_fma(double* out, long long* cyc, int iters, double a, double b) {
  double v[C];
#pragma unroll
  for (int i = 0; i < C; ++i) v[i] = threadIdx.x * 1e-3 + i;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < C; ++i) v[i] = fma(v[i], a, b);
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int C>
__global__ void chain_mul(double* out, long long* cyc, int iters, double a, double b) {
  double v[C];
#pragma unroll
  for (int i = 0; i < C; ++i) v[i] = threadIdx.x * 1e-3 + i + 1.0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < C; ++i) v[i] = v[i] * a + b;
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x * 8] = t1 - t0;
}

template <int C>
__global__ void chain_sqrt(double* out, long long* cyc, int iters, double a, double b) {
  double v[C];
#pragma unroll
  for (int i = 0; i < C; ++i) v[i] = threadIdx.x * 1e-3 + i + 2.0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < C; ++i) v[i] = sqrt(v[i]) + b;
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x * 8] = t1 - t0;
}

template <int C>
__global__ void chain_div(double* out, long long* cyc, int iters, double a, double b) {
  double v[C];
#pragma unroll
  for (int i = 0; i < C; ++i) v[i] = threadIdx.x * 1e-3 + i + 2.0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < C; ++i) v[i] = a / v[i] + b;
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x * 8] = t1 - t0;
}

template <int C>
__global__ void chain_sincos(double* out, long long* cyc, int iters, double a, double b) {
  double v[C];
#pragma unroll
  for (int i = 0; i < C; ++i) v[i] = threadIdx.x * 1e-3 + i + 0.5;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < C; ++i) {
        double s, c;
        sincos(v[i], &s, &c);
        v[i] = s + c * a;
      }
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x * 8] = t1 - t0;
}

typedef void (*K)(double*, long long*, int, double, double);

static void run(const char* name, K k, int chains, int ops_per_iter_chain, double* d_out,
                long long* d_cyc, int blocks, int threads) {
  const int iters = 64;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, iters, 0.999, 1e-3);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, iters, 0.999, 1e-3);
  hipDeviceSynchronize();
  long long c[8];
  hipMemcpy(c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
  const double ops = (double)iters * 16 * ops_per_iter_chain;
  printf("%-8s chains=%d blocks=%d threads=%d: %.2f cycles per dependent op, %.2f per op issued\n",
         name, chains, blocks, threads, c[0] / ops, c[0] / (ops * chains));
}

int main() {
  double* d_out;
  long long* d_cyc;
  hipMalloc(&d_out, 1 << 24);
  hipMalloc(&d_cyc, 1 << 16);
  run("fma", chain_fma<1>, 1, 1, d_out, d_cyc, 1, 64);
  run("fma", chain_fma<2>, 2, 1, d_out, d_cyc, 1, 64);
  run("fma", chain_fma<4>, 4, 1, d_out, d_cyc, 1, 64);
  run("fma", chain_fma<8>, 8, 1, d_out, d_cyc, 1, 64);
  run("fma", chain_fma<1>, 1, 1, d_out, d_cyc, 1, 256);
  run("fma", chain_fma<1>, 1, 1, d_out, d_cyc, 1, 512);
  run("fma", chain_fma<4>, 4, 1, d_out, d_cyc, 1, 512);
  run("fma", chain_fma<1>, 1, 1, d_out, d_cyc, 256, 256);
  run("fma", chain_fma<1>, 1, 1, d_out, d_cyc, 1024, 256);
  run("fma", chain_fma<1>, 1, 1, d_out, d_cyc, 1, 32);
  run("mul+add", chain_mul<1>, 1, 2, d_out, d_cyc, 1, 64);
  run("mul+add", chain_mul<4>, 4, 2, d_out, d_cyc, 1, 64);
  run("sqrt", chain_sqrt<1>, 1, 1, d_out, d_cyc, 1, 64);
  run("sqrt", chain_sqrt<4>, 4, 1, d_out, d_cyc, 1, 64);
  run("div", chain_div<1>, 1, 1, d_out, d_cyc, 1, 64);
  run("div", chain_div<4>, 4, 1, d_out, d_cyc, 1, 64);
  run("sincos", chain_sincos<1>, 1, 1, d_out, d_cyc, 1, 64);
  run("sincos", chain_sincos<4>, 4, 1, d_out, d_cyc, 1, 64);
  return 0;
}
