// LDS throughput probe (timing experiment only, not product code): the cost
// of the per-pixel LDS operations a K1 design can use, at random addresses
// as a uniform image produces them.  Each thread draws pseudo-random slots
// and issues one operation per draw; the kernel runs 2 x 512-thread blocks
// per CU (the production K1 shape) and reports LDS cycles per wave-instruction
// from the wall time.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_probe tools/lds_probe.hip
//   tools/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

enum Op { RD_U8, RD_B64, RD_B128, ADD_U32, ADD_U64, ADD_F64, ADD_F64_PAIR, ADD_U32_F64_F64, NONE };

template <int OP>
__global__ __launch_bounds__(512, 4) void probe(int iters, int nslot, int cshift, unsigned seed, double* sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    for (int i = tid; i < 76 * 1024 / 4; i += 512) reinterpret_cast<unsigned*>(smem)[i] = i;
    __syncthreads();
    unsigned x = seed ^ (tid * 0x9E3779B9u) ^ (blockIdx.x * 0x85EBCA6Bu);
    const int C = 1 << cshift, copy = tid & (C - 1);
    double acc = 0;
    unsigned long long accu = 0;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
#pragma unroll
            for (int q = 0; q < 4; q++) {                       // 4 operations per draw, 8 bits each
                const unsigned b = (x >> (8 * q)) & 255u;
                const int s = (int)((b * (unsigned)nslot) >> 8);   // slot in [0, nslot)
                const int slot = (s << cshift) | copy;
                if constexpr (OP == RD_U8) accu += smem[(slot * 131) & 32767];
                else if constexpr (OP == RD_B64) acc += reinterpret_cast<const double*>(smem)[slot & 4095];
                else if constexpr (OP == RD_B128) {
                    const double2 v = reinterpret_cast<const double2*>(smem)[slot & 2047];
                    acc += v.x + v.y;
                } else if constexpr (OP == ADD_U32) atomicAdd(reinterpret_cast<unsigned*>(smem) + slot, b);
                else if constexpr (OP == ADD_U64) atomicAdd(reinterpret_cast<unsigned long long*>(smem) + slot, (unsigned long long)b);
                else if constexpr (OP == ADD_F64) atomicAdd(reinterpret_cast<double*>(smem) + slot, (double)b);
                else if constexpr (OP == ADD_F64_PAIR) {
                    double* a = reinterpret_cast<double*>(smem) + 2 * slot;
                    atomicAdd(a, (double)b);
                    atomicAdd(a + 1, (double)q);
                } else if constexpr (OP == ADD_U32_F64_F64) {
                    atomicAdd(reinterpret_cast<unsigned*>(smem) + slot, b);
                    double* a = reinterpret_cast<double*>(smem + 16384) + 2 * slot;
                    atomicAdd(a, (double)b);
                    atomicAdd(a + 1, (double)q);
                } else accu += b;
            }
        }
    }
    if (acc == 1.2345 || accu == 12345) sink[0] = acc + accu;
}

template <int OP>
float run(const char* name, int nslot, int cshift, int nops_per_draw) {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    double* sink;
    CK(hipMalloc(&sink, 8));
    CK(hipFuncSetAttribute((const void*)probe<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
    const int iters = 2000, grid = 2 * cus;
    const size_t lds = 76 * 1024;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    probe<OP><<<grid, 512, lds>>>(iters / 10, nslot, cshift, 1, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    probe<OP><<<grid, 512, lds>>>(iters, nslot, cshift, 2, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    // wave-instructions per CU: 16 waves x iters x 8 draws x ops per draw
    const double wi = 16.0 * iters * 8 * nops_per_draw;
    const double cyc = ms * 1e-3 * 2.1e9;                    // at ~2.1 GHz under load
    printf("%-22s nslot %5d copies %2d: %8.3f ms  %6.2f cycles/wave-op (2.1 GHz)  %6.2f per draw\n", name, nslot,
           1 << cshift, ms, cyc / wi, cyc / (16.0 * iters * 8));
    CK(hipFree(sink));
    return ms;
}

int main() {
    run<NONE>("none (xorshift only)", 577, 0, 1);
    run<RD_U8>("ds_read_u8 32KB", 256, 0, 1);
    run<RD_B64>("ds_read_b64 256", 256, 0, 1);
    run<RD_B64>("ds_read_b64 4096", 4096, 0, 1);
    run<RD_B128>("ds_read_b128 256", 256, 0, 1);
    for (int cs = 0; cs <= 5; cs++) run<ADD_U32>("ds_add_u32", 577, cs, 1);
    for (int cs = 0; cs <= 4; cs++) run<ADD_U64>("ds_add_u64", 577, cs, 1);
    for (int cs = 0; cs <= 4; cs++) run<ADD_F64>("ds_add_f64", 113, cs, 1);
    for (int cs = 0; cs <= 4; cs++) run<ADD_F64_PAIR>("ds_add_f64 x2 (h,s)", 113, cs, 2);
    run<ADD_U32>("ds_add_u32 same slot", 1, 0, 1);
    run<ADD_U64>("ds_add_u64 same slot", 1, 0, 1);
    run<ADD_F64>("ds_add_f64 same slot", 1, 0, 1);
    run<ADD_U32>("ds_add_u32 same, 8cp", 1, 3, 1);
    return 0;
}
