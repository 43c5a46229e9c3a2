// Gather floor of the propagation hop (not product code): how fast can the
// frontier rows of a random connectSome overlay be pulled, per node, with no
// other work?  Compares the hop kernel's access shapes:
//   N1  thread per node, U pairs' rows in flight, W = 4 (256 messages)
//   N4  4 lanes per node, a 32-B chunk each, W = 16 (1024 messages)
//   P1  lane per pair (pairs coalesced), W = 4, result per pair
//   S1  N1 over the same overlay renumbered in BFS order (locality)
//   W1  one-word rows (64-message batches): thread per node, LPN lanes per
//       node splitting its pairs (k_prop_hop_fast1's shape), lane per pair;
//       random and BFS order
// Every variant ORs the gathered rows and writes one row per node (or pair),
// so the loads stay live.  Half the pairs are "not in mesh" (pin = NONE).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <queue>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

constexpr uint32_t NONE = 0xFFFFFFFFu;

template <int W, int U>
__global__ __launch_bounds__(256) void k_node(const int64_t* __restrict__ rp, const uint32_t* __restrict__ pin,
                                              const uint64_t* __restrict__ front, uint64_t* __restrict__ nxt,
                                              uint32_t n) {
    for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < n; u += gridDim.x * 256) {
        const int64_t q0 = rp[u], q1 = rp[u + 1];
        uint64_t acc[W] = {};
        for (int64_t qb = q0; qb < q1; qb += U) {
            uint32_t p[U];
#pragma unroll
            for (int j = 0; j < U; ++j) p[j] = qb + j < q1 ? pin[qb + j] : NONE;
            uint64_t c[U][W];
#pragma unroll
            for (int j = 0; j < U; ++j)
#pragma unroll
                for (int i = 0; i < W; ++i) c[j][i] = p[j] != NONE ? front[(size_t)p[j] * W + i] : 0;
#pragma unroll
            for (int j = 0; j < U; ++j)
#pragma unroll
                for (int i = 0; i < W; ++i) acc[i] |= c[j][i];
        }
#pragma unroll
        for (int i = 0; i < W; ++i) nxt[(size_t)u * W + i] = acc[i];
    }
}

// LPN lanes per node, CW words each (W = LPN * CW)
template <int CW, int LPN, int U>
__global__ __launch_bounds__(256) void k_group(const int64_t* __restrict__ rp, const uint32_t* __restrict__ pin,
                                               const uint64_t* __restrict__ front, uint64_t* __restrict__ nxt,
                                               uint32_t n) {
    constexpr int W = CW * LPN;
    const uint32_t lc = threadIdx.x % LPN;
    for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t / LPN < n; t += gridDim.x * 256) {
        const uint32_t u = t / LPN;
        const int64_t q0 = rp[u], q1 = rp[u + 1];
        uint64_t acc[CW] = {};
        for (int64_t qb = q0; qb < q1; qb += U) {
            uint32_t p[U];
#pragma unroll
            for (int j = 0; j < U; ++j) p[j] = qb + j < q1 ? pin[qb + j] : NONE;
            uint64_t c[U][CW];
#pragma unroll
            for (int j = 0; j < U; ++j)
#pragma unroll
                for (int i = 0; i < CW; ++i) c[j][i] = p[j] != NONE ? front[(size_t)p[j] * W + lc * CW + i] : 0;
#pragma unroll
            for (int j = 0; j < U; ++j)
#pragma unroll
                for (int i = 0; i < CW; ++i) acc[i] |= c[j][i];
        }
#pragma unroll
        for (int i = 0; i < CW; ++i) nxt[(size_t)u * W + lc * CW + i] = acc[i];
    }
}

// LPN lanes per node, each taking every LPN-th pair of the row; the lanes'
// ORs are combined with shuffles (one-word rows: the pairs are split, not the row)
template <int LPN, int U>
__global__ __launch_bounds__(256) void k_split1(const int64_t* __restrict__ rp, const uint32_t* __restrict__ pin,
                                               const uint64_t* __restrict__ front, uint64_t* __restrict__ nxt,
                                               uint32_t n) {
    const uint32_t lc = threadIdx.x % LPN;
    for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t / LPN < n; t += gridDim.x * 256) {
        const uint32_t u = t / LPN;
        const int64_t q0 = rp[u], q1 = rp[u + 1];
        uint64_t acc = 0;
        for (int64_t qb = q0 + lc; qb < q1; qb += LPN * U) {
            uint32_t p[U];
#pragma unroll
            for (int j = 0; j < U; ++j) p[j] = qb + j * LPN < q1 ? pin[qb + j * LPN] : NONE;
            uint64_t c[U];
#pragma unroll
            for (int j = 0; j < U; ++j) c[j] = p[j] != NONE ? front[p[j]] : 0;
#pragma unroll
            for (int j = 0; j < U; ++j) acc |= c[j];
        }
#pragma unroll
        for (int o = 1; o < LPN; o <<= 1) acc |= __shfl_xor(acc, o, LPN);
        if (lc == 0) nxt[u] = acc;
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_pair(const uint32_t* __restrict__ pin, const uint64_t* __restrict__ front,
                                              uint64_t* __restrict__ out, uint64_t E) {
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < E; q += (uint64_t)gridDim.x * 256) {
        const uint32_t p = pin[q];
        uint64_t a = 0;
        if (p != NONE)
#pragma unroll
            for (int i = 0; i < W; ++i) a |= front[(size_t)p * W + i];
        if (a == 0x12345) out[q] = a;  // practically never: the loads stay live without a write stream
    }
}

struct Overlay {
    std::vector<int64_t> rp;
    std::vector<uint32_t> col;
};

static Overlay connect_some(uint32_t n, int d, uint64_t seed) {
    std::vector<std::vector<uint32_t>> adj(n);
    uint64_t x = seed;
    auto rnd = [&]() {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < d; ++k) {
            uint32_t j = rnd() % n;
            if (j == i) continue;
            adj[i].push_back(j);
            adj[j].push_back(i);
        }
    Overlay o;
    o.rp.assign(n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) {
        auto& a = adj[i];
        std::sort(a.begin(), a.end());
        a.erase(std::unique(a.begin(), a.end()), a.end());
        o.rp[i + 1] = o.rp[i] + (int64_t)a.size();
    }
    o.col.resize(o.rp[n]);
    for (uint32_t i = 0; i < n; ++i) std::copy(adj[i].begin(), adj[i].end(), o.col.begin() + o.rp[i]);
    return o;
}

static Overlay renumber_bfs(const Overlay& o, uint32_t n) {
    std::vector<uint32_t> order, perm(n, NONE);
    order.reserve(n);
    for (uint32_t s = 0; s < n; ++s) {
        if (perm[s] != NONE) continue;
        std::queue<uint32_t> qu;
        qu.push(s);
        perm[s] = (uint32_t)order.size();
        order.push_back(s);
        while (!qu.empty()) {
            uint32_t v = qu.front();
            qu.pop();
            for (int64_t e = o.rp[v]; e < o.rp[v + 1]; ++e) {
                uint32_t w = o.col[e];
                if (perm[w] == NONE) {
                    perm[w] = (uint32_t)order.size();
                    order.push_back(w);
                    qu.push(w);
                }
            }
        }
    }
    Overlay r;
    r.rp.assign(n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) r.rp[i + 1] = r.rp[i] + (o.rp[order[i] + 1] - o.rp[order[i]]);
    r.col.resize(o.col.size());
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t v = order[i];
        std::vector<uint32_t> nb;
        for (int64_t e = o.rp[v]; e < o.rp[v + 1]; ++e) nb.push_back(perm[o.col[e]]);
        std::sort(nb.begin(), nb.end());
        std::copy(nb.begin(), nb.end(), r.col.begin() + r.rp[i]);
    }
    return r;
}

template <typename F>
static float time_it(F f, int reps = 10) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;  // us
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000;
    Overlay ov = connect_some(n, 6, 42);
    const uint64_t E = ov.rp[n];
    printf("n=%u E=%llu\n", n, (unsigned long long)E);
    for (int order = 0; order < 2; ++order) {
        Overlay o = order ? renumber_bfs(ov, n) : ov;
        std::vector<uint32_t> pin(E);
        uint64_t x = 7;
        for (uint64_t q = 0; q < E; ++q) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            pin[q] = (x >> 63) ? o.col[q] : NONE;  // half in mesh
        }
        int64_t* d_rp;
        uint32_t* d_pin;
        uint64_t *d_front, *d_nxt;
        const int WMAX = 16;
        CHK(hipMalloc(&d_rp, 8 * (n + 1)));
        CHK(hipMalloc(&d_pin, 4 * E));
        CHK(hipMalloc(&d_front, 8ull * WMAX * n));
        CHK(hipMalloc(&d_nxt, 8ull * WMAX * std::max<uint64_t>(n, E)));
        CHK(hipMemcpy(d_rp, o.rp.data(), 8 * (n + 1), hipMemcpyHostToDevice));
        CHK(hipMemcpy(d_pin, pin.data(), 4 * E, hipMemcpyHostToDevice));
        CHK(hipMemset(d_front, 0x5A, 8ull * WMAX * n));
        const dim3 B(256);
        auto grid = [](uint64_t t) { return dim3((unsigned)std::min<uint64_t>((t + 255) / 256, 2048)); };
        const uint64_t mesh = E / 2;
        auto report = [&](const char* name, float us, int W) {
            const double gb = (double)mesh * W * 8 / 1e9;
            printf("%s %-22s %8.1f us  %6.1f GB/s of row bytes (%d words)\n", order ? "bfs " : "rand", name, us,
                   gb / (us * 1e-6), W);
        };
        report("node W1 U4", time_it([&] { k_node<1, 4><<<grid(n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 1);
        report("node W1 U8", time_it([&] { k_node<1, 8><<<grid(n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 1);
        report("split W1 lpn4 U2", time_it([&] { k_split1<4, 2><<<grid(4ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 1);
        report("split W1 lpn4 U1", time_it([&] { k_split1<4, 1><<<grid(4ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 1);
        report("split W1 lpn8 U1", time_it([&] { k_split1<8, 1><<<grid(8ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 1);
        report("pair W1", time_it([&] { k_pair<1><<<grid(E), B>>>(d_pin, d_front, d_nxt, E); }), 1);
        if (!order) {  // (the BFS order only for one-word rows)
        report("node W4 U4", time_it([&] { k_node<4, 4><<<grid(n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 4);
        report("node W4 U8", time_it([&] { k_node<4, 8><<<grid(n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 4);
        report("node W4 U2", time_it([&] { k_node<4, 2><<<grid(n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 4);
        report("group W4 cw1 lpn4", time_it([&] { k_group<1, 4, 4><<<grid(4ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 4);
        report("group W4 cw2 lpn2", time_it([&] { k_group<2, 2, 4><<<grid(2ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 4);
        report("group W16 cw4 lpn4", time_it([&] { k_group<4, 4, 4><<<grid(4ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 16);
        report("group W16 cw2 lpn8", time_it([&] { k_group<2, 8, 4><<<grid(8ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 16);
        report("group W16 cw4 lpn4 U8", time_it([&] { k_group<4, 4, 8><<<grid(4ull * n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 16);
        report("node W16 U2", time_it([&] { k_node<16, 2><<<grid(n), B>>>(d_rp, d_pin, d_front, d_nxt, n); }), 16);
        for (int lds : {20 * 1024, 40 * 1024, 80 * 1024}) {  // limits blocks per CU: 8, 4, 2 (of 160 KB)
            char nm[64];
            snprintf(nm, sizeof nm, "group W16 lds%dK", lds / 1024);
            report(nm, time_it([&] { hipLaunchKernelGGL((k_group<4, 4, 4>), grid(4ull * n), B, lds, 0, d_rp, d_pin, d_front, d_nxt, n); }), 16);
            snprintf(nm, sizeof nm, "node W4 lds%dK", lds / 1024);
            report(nm, time_it([&] { hipLaunchKernelGGL((k_node<4, 4>), grid(n), B, lds, 0, d_rp, d_pin, d_front, d_nxt, n); }), 4);
        }
        report("pair W4", time_it([&] { k_pair<4><<<grid(E), B>>>(d_pin, d_front, d_nxt, E); }), 4);
        report("pair W16", time_it([&] { k_pair<16><<<grid(E), B>>>(d_pin, d_front, d_nxt, E); }), 16);
        }
        CHK(hipFree(d_rp));
        CHK(hipFree(d_pin));
        CHK(hipFree(d_front));
        CHK(hipFree(d_nxt));
    }
    return 0;
}
