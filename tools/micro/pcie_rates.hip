// Host<->device transfer rates on the box: pageable vs registered vs hipHostMalloc'd buffers (sizes of C4's band
// and arena), and the cost of pinning.  Informs the host-pointer encode path (DESIGN.md "End to end").
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main(int argc, char **argv) {
    const size_t n = (argc > 1 ? atoll(argv[1]) : 3200) * (size_t)1000000;
    void *d;
    CK(hipMalloc(&d, n));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    char *pg = (char *)malloc(n);
    memset(pg, 1, n);
    double t = now();
    CK(hipMemcpyAsync(d, pg, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
    printf("pageable H2D  %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(pg, d, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s));
    printf("pageable D2H  %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipHostRegister(pg, n, hipHostRegisterDefault));
    printf("register      %.3f s (%.1f GB/s)\n", now() - t, n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(d, pg, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
    printf("registered H2D %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(pg, d, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s));
    printf("registered D2H %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipHostUnregister(pg));
    printf("unregister    %.3f s\n", now() - t);
    char *hp;
    t = now();
    CK(hipHostMalloc((void **)&hp, n, hipHostMallocDefault));
    printf("hipHostMalloc %.3f s\n", now() - t);
    t = now();
    memset(hp, 2, n);
    printf("memset pinned %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
    printf("pinned H2D    %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(hp, d, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s));
    printf("pinned D2H    %.1f GB/s\n", n / (now() - t) / 1e9);
    // both directions at once on two streams
    hipStream_t s2;
    CK(hipStreamCreate(&s2));
    void *d2;
    CK(hipMalloc(&d2, n));
    t = now();
    CK(hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(pg, d2, n, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s)); CK(hipStreamSynchronize(s2));
    printf("H2D(pinned)+D2H(pageable) concurrent %.3f s\n", now() - t);
    t = now();
    memcpy(pg, hp, n);
    printf("host memcpy   %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    FILE *f = fopen(getenv("OUTF") ? getenv("OUTF") : "/tmp/pcie_rates.bin", "wb");
    fwrite(hp, 1, n, f);
    fclose(f);
    printf("file write    %.1f GB/s\n", n / (now() - t) / 1e9);
    remove(getenv("OUTF") ? getenv("OUTF") : "/tmp/pcie_rates.bin");
    return 0;
}
