// Exhaustive check (every finite normal float with 2^-125 <= |x| < 2^125) that
// one FMA Newton step on the hardware reciprocal gives the IEEE correctly
// rounded 1/x bit for bit:  r = rcp(x); e = fma(-x, r, 1); r' = fma(e, r, r).
// Used to justify pm_device.h rcp_exact(). Prints mismatch count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(unsigned long long *bad, uint32_t *first) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long nb = 0;
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t bits = (uint32_t)(tid * 16 + k);
        const uint32_t ex = (bits >> 23) & 0xffu;
        if (ex < 2 || ex > 251) continue; /* |x| in [2^-125, 2^125) */
        const float x = __uint_as_float(bits);
        const float ieee = __fdiv_rn(1.0f, x);
        const float r = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, r, 1.0f);
        const float r1 = __builtin_fmaf(e, r, r);
        if (__float_as_uint(r1) != __float_as_uint(ieee)) {
            ++nb;
            atomicMin(first, bits);
        }
    }
    if (nb) atomicAdd(bad, nb);
}

int main() {
    unsigned long long *bad; uint32_t *first;
    (void)hipMalloc(&bad, 8); (void)hipMalloc(&first, 4);
    (void)hipMemset(bad, 0, 8); (void)hipMemset(first, 0xff, 4);
    const uint64_t total = 1ull << 32, per = 16, threads = total / per;
    hipLaunchKernelGGL(check, dim3((unsigned)(threads / 256)), dim3(256), 0, 0, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    unsigned long long hb; uint32_t hf;
    (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    printf("mismatches %llu first 0x%08x\n", hb, hf);
    return hb ? 1 : 0;
}
