// Calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the engine uses (MI355X_MICROARCH.md: "calibrate on a known byte
// count in your own access pattern before trusting an absolute").
// Each kernel streams exactly BYTES bytes; compare the counters with BYTES.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t BYTES = size_t(1) << 30;  // 1 GiB, far beyond the 256 MiB Infinity Cache

template <typename V>
__global__ __launch_bounds__(256) void k_read(const V* __restrict__ a, size_t n, double* out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    double s = 0;
    for (; i < n; i += (size_t)gridDim.x * 256) {
        const V v = a[i];
        s += (double)(reinterpret_cast<const unsigned char*>(&v)[0]);
    }
    if (s == -1.0) out[0] = s;  // keep the loads live, never true
}

template <typename V>
__global__ __launch_bounds__(256) void k_write(V* __restrict__ a, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * 256) a[i] = V{};
}

__global__ __launch_bounds__(256) void k_read_u8(const unsigned char* __restrict__ a, size_t n, double* out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    double s = 0;
    for (; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    if (s == -1.0) out[0] = s;
}

int main() {
    void* buf;
    double* out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    hipMemset(buf, 1, BYTES);
    const int grid = 256 * 8;
    for (int rep = 0; rep < 2; ++rep) {
        k_read<double><<<grid, 256>>>((const double*)buf, BYTES / 8, out);      // 8 B per lane
        k_read<double2><<<grid, 256>>>((const double2*)buf, BYTES / 16, out);   // 16 B per lane
        k_read_u8<<<grid, 256>>>((const unsigned char*)buf, BYTES, out);        // 1 B per lane
        k_write<double><<<grid, 256>>>((double*)buf, BYTES / 8);
        k_write<double2><<<grid, 256>>>((double2*)buf, BYTES / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("each kernel streams %zu bytes\n", BYTES);
    return 0;
}
