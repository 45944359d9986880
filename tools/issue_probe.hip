// issue_probe.hip -- design probe (not product code): does a CU issue VALU
// and SALU instructions in the same cycle?  The hint kernel issues ~0.99
// instructions per CU per cycle (VALU 0.68 + SALU 0.28 + LDS/VMEM), the ACL
// kernel 0.77, while neither VALU nor SALU alone is near its own peak
// (scripts/sq_summary.py).  Each kernel below runs a fixed loop of
// independent instructions at 8 waves per SIMD:
//   valu:      8 v_add_u32 per iteration (4 independent chains x 2)
//   valu_salu: the same 8 plus 4 s_add_u32 (2 scalar chains x 2)
//   salu:      4 s_add_u32 only
// and reports wave-instructions per CU per cycle, the cycle count taken
// in-kernel (s_memtime over s_memrealtime at 100 MHz).
//
//   hipcc -O3 --offload-arch=gfx950 tools/issue_probe.hip -o tools/issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

constexpr int kIters = 20000;

template <int kMode>   // 0 valu, 1 valu+salu, 2 salu
__global__ __launch_bounds__(256) void probe(uint32_t* out, unsigned long long* clk) {
    uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    uint32_t s0 = blockIdx.x, s1 = s0 + 7;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < kIters; ++i) {
        if (kMode != 2)
            asm volatile(
                "v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\t"
                "v_add_u32 %3, %3, %4\n\tv_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\t"
                "v_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4"
                : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
                : "v"(threadIdx.x));
        if (kMode != 0)
            asm volatile(
                "s_add_u32 %0, %0, 3\n\ts_add_u32 %1, %1, 5\n\ts_add_u32 %0, %0, 3\n\t"
                "s_add_u32 %1, %1, 5"
                : "+s"(s0), "+s"(s1)
                :
                : "scc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + s0 + s1;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int grid = cus * 8;                 // 8 x 4 waves = 8 waves per SIMD
    uint32_t* out;
    unsigned long long *clk, h[2];
    CK(hipMalloc(&out, size_t(grid) * 256 * 4));
    CK(hipMalloc(&clk, 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[3] = {"valu", "valu_salu", "salu"};
    const int valu[3] = {8, 8, 0}, salu[3] = {0, 4, 4};
    printf("mode,ms,clock_GHz,valu_per_cu_cycle,salu_per_cu_cycle,all_per_cu_cycle\n");
    for (int m = 0; m < 3; ++m)
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, 0));
            if (m == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, out, clk);
            if (m == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, out, clk);
            if (m == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, out, clk);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
            const double ghz = double(h[0]) / (double(h[1]) / 100e6) / 1e9;
            const double cycles = ms * 1e-3 * ghz * 1e9;
            const double waves = double(grid) * 4;
            const double v = waves * kIters * valu[m] / cus / cycles;
            const double s = waves * kIters * salu[m] / cus / cycles;
            if (rep > 0) printf("%s,%.3f,%.2f,%.3f,%.3f,%.3f\n", names[m], ms, ghz, v, s, v + s);
        }
    return 0;
}
