// Probe: does v_mad_u16 with op_sel (high half of src2) clear the upper 16
// bits of its destination on gfx950?  Prints the result for a destination
// register that held 0xFFFF0000 before.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(unsigned* o, unsigned a, unsigned e) {
    unsigned r = 0xFFFF0000u + threadIdx.x * 0u;
    asm volatile("v_mad_u16 %0, %1, 4, %2 op_sel:[0,0,1,0]" : "+v"(r) : "v"(a), "v"(e));
    o[threadIdx.x] = r;
}

int main() {
    unsigned* d;
    hipMalloc(&d, 64 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 5u, 0x01230000u | 0x1234u);
    unsigned h[64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mad_u16 op_sel result 0x%08x (expect low half 0x%04x)\n", h[0], (5u * 4u + 0x0123u) & 0xFFFFu);
    return 0;
}
