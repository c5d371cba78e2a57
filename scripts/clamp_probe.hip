// Probe: semantics of v_pk_mul_lo_u16 with the clamp bit on gfx950 (2048 * 32 per half) — ignored —
// and of the saturating v_pk_add_u16 clamp the composite's weights rely on instead.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o, unsigned a, unsigned b) {
    unsigned r, q, s;
    asm volatile("v_pk_mul_lo_u16 %0, %1, %2 op_sel_hi:[1,0] clamp" : "=v"(r) : "v"(a), "v"(b));
    asm volatile("v_pk_mul_lo_u16 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(q) : "v"(a), "v"(b));
    asm volatile("v_pk_add_u16 %0, %1, %2 clamp" : "=v"(s) : "v"(a * 31u), "v"(a));  // 31a + a, saturating
    if (threadIdx.x == 0) { o[0] = r; o[1] = q; o[2] = s; }
}
int main() {
    unsigned* d; unsigned h[3];
    hipMalloc(&d, 12);
    const unsigned tests[][2] = {{2048u, 32u}, {(64u << 16) | 1984u, 31u}, {(1984u << 16) | 64u, 32u}, {2048u, 0u}};
    for (auto& t : tests) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, t[0], t[1]);
        hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
        printf("a=%08x b=%u clamp=%08x plain=%08x add_sat(31a, a)=%08x\n", t[0], t[1], h[0], h[1], h[2]);
    }
    return 0;
}
