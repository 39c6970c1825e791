// tools/perf_group.h — hardware counters (user space, this thread) for the
// host-walk benches (RB_PERF=1 in tools/replay_bench and tools/range_bench):
// cycles, instructions, branch misses, L1D read misses — where the host
// exposes a PMU (the GPU boxes; not this build container).
#pragma once
#include <cstdint>
#include <cstring>
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <unistd.h>

struct PerfGroup {
    int fd[4] = {-1, -1, -1, -1};
    uint64_t v[4] = {};
    static int open1(uint32_t type, uint64_t config) {
        perf_event_attr a;
        std::memset(&a, 0, sizeof a);
        a.type = type;
        a.size = sizeof a;
        a.config = config;
        a.disabled = 1;
        a.exclude_kernel = 1;
        a.exclude_hv = 1;
        return (int)syscall(__NR_perf_event_open, &a, 0, -1, -1, 0);
    }
    PerfGroup() {
        fd[0] = open1(PERF_TYPE_HARDWARE, PERF_COUNT_HW_CPU_CYCLES);
        fd[1] = open1(PERF_TYPE_HARDWARE, PERF_COUNT_HW_INSTRUCTIONS);
        fd[2] = open1(PERF_TYPE_HARDWARE, PERF_COUNT_HW_BRANCH_MISSES);
        fd[3] = open1(PERF_TYPE_HW_CACHE, PERF_COUNT_HW_CACHE_L1D | (PERF_COUNT_HW_CACHE_OP_READ << 8) |
                                              (PERF_COUNT_HW_CACHE_RESULT_MISS << 16));
    }
    ~PerfGroup() {
        for (int k = 0; k < 4; k++)
            if (fd[k] >= 0) close(fd[k]);
    }
    bool ok() const { return fd[0] >= 0; }
    void start() {
        for (int k = 0; k < 4; k++)
            if (fd[k] >= 0) { ioctl(fd[k], PERF_EVENT_IOC_RESET, 0); ioctl(fd[k], PERF_EVENT_IOC_ENABLE, 0); }
    }
    void stop() {
        for (int k = 0; k < 4; k++) {
            if (fd[k] < 0) continue;
            ioctl(fd[k], PERF_EVENT_IOC_DISABLE, 0);
            uint64_t x = 0;
            if (read(fd[k], &x, sizeof x) == (ssize_t)sizeof x) v[k] += x;
        }
    }
};
