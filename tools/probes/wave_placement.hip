// Probe: which SIMD does each wave of a 320-thread (5-wave) workgroup land on, and how do co-resident
// workgroups of one CU spread?  Reads HW_REG_HW_ID (wave, SIMD, CU, SE) and HW_REG_XCC_ID per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <map>
#include <tuple>

__global__ void __launch_bounds__(320) probe(unsigned *out, int spin)
{
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // keep the workgroup resident a while so co-residency is visible
    long t0 = clock64();
    while (clock64() - t0 < spin) {}
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        out[(blockIdx.x * 5 + w) * 2] = hw;
        out[(blockIdx.x * 5 + w) * 2 + 1] = xcc;
    }
}

int main()
{
    const int B = 1024;
    unsigned *d;
    hipMalloc(&d, sizeof(unsigned) * B * 10);
    hipLaunchKernelGGL(probe, dim3(B), dim3(320), 0, 0, d, 200000);
    std::vector<unsigned> h(B * 10);
    hipMemcpy(h.data(), d, sizeof(unsigned) * B * 10, hipMemcpyDeviceToHost);
    // per block: SIMD of each wave; histogram of wave-4 SIMD, and per (xcc, se, cu) the blocks + their wave-4 SIMDs
    int hist[5][4] = {};
    std::map<std::tuple<int, int, int>, std::vector<std::pair<int, int>>> cu;
    for (int b = 0; b < B; ++b)
        for (int w = 0; w < 5; ++w) {
            const unsigned hw = h[(b * 5 + w) * 2], xcc = h[(b * 5 + w) * 2 + 1] & 0xF;
            const int simd = (hw >> 4) & 3, cuid = (hw >> 8) & 15, se = (hw >> 13) & 7;
            hist[w][simd]++;
            if (w == 4) cu[{(int)xcc, se, cuid}].push_back({b, simd});
        }
    for (int w = 0; w < 5; ++w) printf("wave %d SIMD histogram: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    int shown = 0;
    for (auto &kv : cu) {
        if (shown++ >= 6) break;
        printf("xcc %d se %d cu %d:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first));
        for (auto &p : kv.second) printf(" (blk %d -> simd %d)", p.first, p.second);
        printf("\n");
    }
    // first block's 5 waves
    for (int b = 0; b < 4; ++b) {
        printf("block %d:", b);
        for (int w = 0; w < 5; ++w) printf(" w%d simd %u", w, (h[(b * 5 + w) * 2] >> 4) & 3);
        printf("\n");
    }
    printf("distinct CUs %zu\n", cu.size());
    return 0;
}
