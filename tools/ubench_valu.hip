// Micro-benchmark: issue throughput of the gfx950 VALU integer/fp64 instructions
// candidate field-arithmetic representations depend on. One asm statement per
// op, 8 independent chains per lane so dependency latency is hidden.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define BODY8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_mul_lo(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_hi(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad_u64(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1, c = seed ^ 0x55;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
    BODY8(S)
#undef S
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_mul_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1, c = seed ^ 7;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add_u32(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_addc_u32(uint32_t* out, uint32_t seed) {
  // v_add_co_u32 + v_addc_co_u32 pairs (64-bit add): counts 2 instructions per pair
  uint32_t a[8], h[8]; for (int i = 0; i < 8; i++) { a[i] = seed + threadIdx.x + i; h[i] = i; }
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS / 2; it++) {
#define S(i) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, 0, vcc" : "+v"(a[i]), "+v"(h[i]) : "v"(b) : "vcc");
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i] ^ h[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma_f64(uint32_t* out, uint32_t seed) {
  double a[8]; for (int i = 0; i < 8; i++) a[i] = (double)(seed + threadIdx.x + i) * 1e-3;
  double b = 0.999999, c = 1e-9;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    BODY8(S)
#undef S
  }
  double s = 0; for (int i = 0; i < 8; i++) s += a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_fma_f32(uint32_t* out, uint32_t seed) {
  float a[8]; for (int i = 0; i < 8; i++) a[i] = (float)(seed + threadIdx.x + i) * 1e-3f;
  float b = 0.999f, c = 1e-6f;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    BODY8(S)
#undef S
  }
  float s = 0; for (int i = 0; i < 8; i++) s += a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_lshl_add(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; it++) {
#define S(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
    BODY8(S)
#undef S
  }
  uint32_t s = 0; for (int i = 0; i < 8; i++) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d clock=%d kHz\n", p.name, p.multiProcessorCount, p.clockRate);
  const int blocks = p.multiProcessorCount * 8, threads = 256;
  uint32_t* out; CHECK(hipMalloc(&out, blocks * threads * 4));
  struct { const char* name; kfn f; double ops_per_iter; } ks[] = {
    {"v_mul_lo_u32", k_mul_lo, 8}, {"v_mul_hi_u32", k_mul_hi, 8}, {"v_mad_u64_u32", k_mad_u64, 8},
    {"v_mul_u32_u24", k_mul_u24, 8}, {"v_mul_hi_u32_u24", k_mulhi_u24, 8}, {"v_mad_u32_u24", k_mad_u24, 8},
    {"v_add_u32", k_add_u32, 8}, {"v_add_co+v_addc (per instr)", k_addc_u32, 8}, {"v_add3_u32", k_lshl_add, 8},
    {"v_fma_f64", k_fma_f64, 8}, {"v_fma_f32", k_fma_f32, 8},
  };
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u + r);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    double lane_ops = 5.0 * blocks * threads * (double)ITERS * k.ops_per_iter;
    double tops = lane_ops / (ms * 1e-3) / 1e12;
    // cycles per wave-instruction per SIMD at 2.4 GHz nominal
    double simds = p.multiProcessorCount * 4.0;
    double wave_instr = lane_ops / 64.0;
    double cyc = (ms * 1e-3) * 2.4e9 * simds / wave_instr;
    printf("%-32s %8.2f T lane-op/s   %5.2f cyc/wave-instr/SIMD (at 2.4GHz)\n", k.name, tops, cyc);
  }
  return 0;
}
