// tools/sweep_bench.cpp — the pass's cold sequential host sweeps over the
// store (assemble's count and scatter, finish's retire) on C3's shape: 1M
// slots, 8 pools, 16 threads one per core of the calling thread's node.
// Variants: as the library writes them, with software prefetch of every
// stream, and with the arrays on transparent huge pages (MADV_HUGEPAGE).
// Each measurement follows an evicting sweep over 256 MB (the arrays are cold,
// as after the Insert that precedes a pass).  Prints per-variant medians.
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static std::vector<int> parse_cpulist(const std::string& path) {
    std::vector<int> out;
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return out;
    char buf[4096];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* p = buf;
    while (*p >= '0' && *p <= '9') {
        char* e;
        const long a = std::strtol(p, &e, 10);
        long b = a;
        p = e;
        if (*p == '-') { b = std::strtol(p + 1, &e, 10); p = e; }
        for (long c = a; c <= b; c++) out.push_back((int)c);
        if (*p == ',') p++;
    }
    return out;
}

template <class T> T* alloc(size_t n, bool huge) {
    const size_t bytes = (n * sizeof(T) + (2u << 20) - 1) & ~((size_t)(2u << 20) - 1);
    void* p = std::aligned_alloc(2u << 20, bytes);
    if (huge) madvise(p, bytes, MADV_HUGEPAGE);
    std::memset(p, 0, bytes);
    return (T*)p;
}

int main(int argc, char** argv) {
    const size_t N = 1u << 20;
    const int P = 8, NT = argc > 1 ? std::atoi(argv[1]) : 16, REPS = 15;
    // one CPU per core of this thread's node
    const int me = sched_getcpu();
    std::vector<int> node;
    for (int nd = 0; nd < 64; nd++) {
        auto l = parse_cpulist("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist");
        if (std::find(l.begin(), l.end(), me) != l.end()) { node = l; break; }
    }
    std::vector<int> cores;
    for (int c : node) {
        auto sib = parse_cpulist("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list");
        if (!sib.empty() && sib[0] == c) cores.push_back(c);
    }
    std::printf("node of cpu %d: %zu cpus, %zu cores; threads %d\n", me, node.size(), cores.size(), NT);
    for (int huge = 0; huge < 2; huge++) {
        uint32_t* rows = alloc<uint32_t>(N, huge);
        uint8_t *sel = alloc<uint8_t>(N, huge), *dec = alloc<uint8_t>(N, huge), *selfm = alloc<uint8_t>(N, huge),
                *idx = alloc<uint8_t>(N, huge), *live = alloc<uint8_t>(N, huge), *act = alloc<uint8_t>(N, huge);
        uint32_t* sig = alloc<uint32_t>(N, huge);
        uint32_t *brow = alloc<uint32_t>(N, huge), *bgrp = alloc<uint32_t>(N, huge), *prow = alloc<uint32_t>(N, huge);
        std::vector<uint8_t> evict(256u << 20, 1);
        for (size_t i = 0; i < N; i++) {
            rows[i] = (uint32_t)i;
            sig[i] = (uint32_t)((i * 2654435761u) >> 29) & 7;
            selfm[i] = idx[i] = live[i] = act[i] = 1;
        }
        for (int pf = 0; pf < 2; pf++) {
            std::vector<double> tc, ts, tr;
            for (int rep = 0; rep < REPS; rep++) {
                for (size_t k = 0; k < evict.size(); k += 64) evict[k]++;
                std::vector<std::vector<uint32_t>> cnt(NT, std::vector<uint32_t>(P, 0));
                auto par = [&](auto fn) {
                    std::vector<std::thread> th;
                    std::atomic<int> go{0};
                    std::vector<double> us(NT);
                    for (int t = 0; t < NT; t++)
                        th.emplace_back([&, t] {
                            cpu_set_t cs;
                            CPU_ZERO(&cs);
                            CPU_SET(cores[(size_t)t % cores.size()], &cs);
                            sched_setaffinity(0, sizeof cs, &cs);
                            go++;
                            while (go.load() < NT) {}
                            auto a = std::chrono::steady_clock::now();
                            fn(t);
                            us[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
                        });
                    for (auto& x : th) x.join();
                    return *std::max_element(us.begin(), us.end());
                };
                tc.push_back(par([&](int t) {
                    uint32_t* c = cnt[t].data();
                    const size_t lo = N * t / NT, hi = N * (t + 1) / NT;
                    bool self = true;
                    for (size_t i = lo; i < hi; i++) {
                        if (pf && (i & 63) == 0) {
                            __builtin_prefetch(rows + i + 512);
                            __builtin_prefetch(sig + i + 512);
                            __builtin_prefetch(sel + i + 2048);
                            __builtin_prefetch(dec + i + 2048);
                            __builtin_prefetch(selfm + i + 2048);
                            __builtin_prefetch(idx + i + 2048);
                            __builtin_prefetch(rows + i + 528);
                            __builtin_prefetch(sig + i + 528);
                        }
                        const uint32_t r = rows[i];
                        if (sel[r] | dec[r]) continue;
                        c[sig[r]]++;
                        self = self & selfm[r] & idx[r];
                    }
                    if (!self) c[0]++;
                }));
                ts.push_back(par([&](int t) {
                    const size_t lo = N * t / NT, hi = N * (t + 1) / NT;
                    uint32_t ga[8];
                    for (int g = 0; g < P; g++) ga[g] = (uint32_t)(g * (N / P) + lo / P);
                    size_t o = lo;
                    for (size_t i = lo; i < hi; i++) {
                        if (pf && (i & 15) == 0) {
                            __builtin_prefetch(rows + i + 256);
                            __builtin_prefetch(sig + i + 256);
                            __builtin_prefetch(brow + i + 256, 1);
                            __builtin_prefetch(bgrp + i + 256, 1);
                        }
                        const uint32_t r = rows[i];
                        if (sel[r] | dec[r]) continue;
                        const uint32_t gi = sig[r];
                        brow[o] = r;
                        bgrp[o] = gi;
                        prow[ga[gi]++] = (uint32_t)o;
                        o++;
                    }
                }));
                for (size_t i = 0; i < N; i++) sel[i] = 1;  // every slot matched (C3)
                for (size_t k = 0; k < evict.size(); k += 64) evict[k]++;
                tr.push_back(par([&](int t) {
                    const size_t lo = N * t / NT, hi = N * (t + 1) / NT;
                    uint32_t k = 0;
                    for (size_t s = lo; s < hi; s++) {
                        if (pf && (s & 63) == 0) {
                            __builtin_prefetch(sel + s + 2048);
                            __builtin_prefetch(live + s + 2048, 1);
                            __builtin_prefetch(act + s + 2048, 1);
                        }
                        if (sel[s] & live[s]) {
                            live[s] = 0;
                            act[s] = 0;
                            k++;
                        }
                    }
                    cnt[t][0] += k;
                }));
                for (size_t i = 0; i < N; i++) { sel[i] = 0; live[i] = act[i] = 1; }
            }
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
            std::printf("huge %d prefetch %d: count %.1f us, scatter %.1f us, retire %.1f us (max over threads, median)\n",
                        huge, pf, med(tc), med(ts), med(tr));
        }
    }
    return 0;
}
