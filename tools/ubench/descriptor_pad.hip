// Compile-only probe (hipcc --cuda-device-only -S): which attributes make hipcc pad
// .amdhsa_next_free_vgpr above the registers a kernel uses (static LDS that
// bounds occupancy, a waves_per_eu maximum).  profiles/r5/coresidency/descriptors.txt
#include <hip/hip_runtime.h>
__global__ __launch_bounds__(1024) void k_static(const unsigned *in, unsigned *out) {
    __shared__ unsigned tbl[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) tbl[i] = in[i];
    __syncthreads();
    out[blockIdx.x * 1024 + threadIdx.x] = tbl[(in[threadIdx.x] & 32767)];
}
__global__ __launch_bounds__(1024) void k_dyn(const unsigned *in, unsigned *out) {
    extern __shared__ unsigned dtbl[];
    for (int i = threadIdx.x; i < 32768; i += 1024) dtbl[i] = in[i];
    __syncthreads();
    out[blockIdx.x * 1024 + threadIdx.x] = dtbl[(in[threadIdx.x] & 32767)];
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_w22(const unsigned *in, unsigned *out) {
    out[threadIdx.x] = in[threadIdx.x] * 3;
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_w2(const unsigned *in, unsigned *out) {
    out[threadIdx.x] = in[threadIdx.x] * 3;
}
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_static_w48(const unsigned *in, unsigned *out) {
    __shared__ unsigned tbl[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) tbl[i] = in[i];
    __syncthreads();
    out[blockIdx.x * 1024 + threadIdx.x] = tbl[(in[threadIdx.x] & 32767)];
}
