// Developer tool: device limits that shape the launch (LDS per block / per CU, CUs).
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
    int v = 0;
#define A(x) (void)hipDeviceGetAttribute(&v, x, 0), printf(#x " = %d\n", v)
    A(hipDeviceAttributeMaxSharedMemoryPerBlock);
    A(hipDeviceAttributeSharedMemPerBlockOptin);
    A(hipDeviceAttributeMaxSharedMemoryPerMultiprocessor);
    A(hipDeviceAttributeMultiprocessorCount);
    A(hipDeviceAttributeClockRate);
    A(hipDeviceAttributeMaxRegistersPerBlock);
    return 0;
}
