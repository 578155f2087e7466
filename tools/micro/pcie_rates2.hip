// Host-side rates for the end-to-end create-streaming pipeline (DESIGN.md "End to end"): pinned staging fed by
// multi-threaded memcpy from pageable memory, DMA rates in both directions (alone and concurrent), the cost of
// pinning in place, and multi-threaded file writes to /dev/shm.  Usage: pcie_rates2 [MB] [threads]
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static void par_copy(char *dst, const char *src, size_t n, int nt) {
    std::vector<std::thread> th;
    const size_t c = (n + nt - 1) / nt;
    for (int i = 0; i < nt; i++) {
        const size_t a = std::min(n, i * c), b = std::min(n, a + c);
        th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
    }
    for (auto &t : th) t.join();
}
int main(int argc, char **argv) {
    const size_t n = (argc > 1 ? atoll(argv[1]) : 3200) * (size_t)1000000;
    const int nt = argc > 2 ? atoi(argv[2]) : 8;
    void *d, *d2;
    CK(hipMalloc(&d, n));
    CK(hipMalloc(&d2, n));
    hipStream_t s, s2;
    CK(hipStreamCreate(&s));
    CK(hipStreamCreate(&s2));
    char *pg = (char *)malloc(n), *pg2 = (char *)malloc(n);
    double t = now();
    par_copy(pg, pg2, n, nt);  // first touch (page faults) of both
    memset(pg, 1, n);
    memset(pg2, 3, n);
    printf("first-touch+memset %.3f s\n", now() - t);
    t = now();
    CK(hipMemcpyAsync(d, pg, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
    printf("pageable H2D  %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(pg, d, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s));
    printf("pageable D2H  %.1f GB/s\n", n / (now() - t) / 1e9);
    char *hp, *hp2;
    t = now();
    CK(hipHostMalloc((void **)&hp, n, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&hp2, n, hipHostMallocDefault));
    printf("hipHostMalloc x2 %.3f s\n", now() - t);
    for (int k : {1, 4, 8, 16}) {
        t = now();
        par_copy(hp, pg, n, k);
        printf("memcpy pageable->pinned, %2d threads  %.1f GB/s\n", k, n / (now() - t) / 1e9);
    }
    t = now();
    CK(hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
    printf("pinned H2D    %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(hp2, d2, n, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s));
    printf("pinned D2H    %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(hp2, d2, n, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s)); CK(hipStreamSynchronize(s2));
    printf("pinned H2D + D2H concurrent: %.1f GB/s each way\n", n / (now() - t) / 1e9);
    // chunked H2D through a 2 x 64 MB pinned ring fed by threaded memcpy (the pageable-source pipeline)
    {
        const size_t ch = 64 << 20;
        hipEvent_t ev[2];
        CK(hipEventCreate(&ev[0]));
        CK(hipEventCreate(&ev[1]));
        bool used[2] = {false, false};
        t = now();
        for (size_t off = 0, i = 0; off < n; off += ch, i++) {
            const size_t m = std::min(ch, n - off);
            const int b = (int)(i & 1);
            if (used[b]) CK(hipEventSynchronize(ev[b]));
            par_copy(hp + b * ch, pg + off, m, nt);
            CK(hipMemcpyAsync((char *)d + off, hp + b * ch, m, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[b], s));
            used[b] = true;
        }
        CK(hipStreamSynchronize(s));
        printf("ring H2D (pageable src, %d threads)  %.1f GB/s\n", nt, n / (now() - t) / 1e9);
    }
    t = now();
    CK(hipHostRegister(pg, n, hipHostRegisterDefault));
    printf("hipHostRegister %.3f s\n", now() - t);
    t = now();
    CK(hipMemcpyAsync(d, pg, n, hipMemcpyHostToDevice, s)); CK(hipStreamSynchronize(s));
    printf("registered H2D %.1f GB/s\n", n / (now() - t) / 1e9);
    t = now();
    CK(hipHostUnregister(pg));
    printf("unregister    %.3f s\n", now() - t);
    const char *fn = getenv("OUTF") ? getenv("OUTF") : "/dev/shm/pcie_rates2.bin";
    for (int k : {1, 4, 8}) {
        t = now();
        int fd = open(fn, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        std::vector<std::thread> th;
        const size_t c = (n + k - 1) / k;
        for (int i = 0; i < k; i++) {
            const size_t a = std::min(n, i * c), b = std::min(n, a + c);
            th.emplace_back([=] {
                size_t o = a;
                while (o < b) {
                    ssize_t w = pwrite(fd, hp + o, std::min<size_t>(b - o, 1 << 30), (off_t)o);
                    if (w <= 0) break;
                    o += (size_t)w;
                }
            });
        }
        for (auto &x : th) x.join();
        close(fd);
        printf("file write %d threads  %.1f GB/s\n", k, n / (now() - t) / 1e9);
        unlink(fn);
    }
    return 0;
}
