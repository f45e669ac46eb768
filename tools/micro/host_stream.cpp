// Streaming-store bandwidth into one host buffer (can the host memory take N GPUs'
// delivered frames?).  A buffer of --mb MiB is first touched by a thread on the process's first
// allowed CPU (so its pages sit on that CPU's NUMA node), then T threads -- each pinned to a CPU of
// its own CPU domain (last-level cache) as far as there are domains, domains on the buffer's node
// first -- write disjoint slices of it with 32-B non-temporal stores, as the library's fill threads
// do.  Best of --reps runs per thread count.
//
// Build: g++ -O2 -mavx2 -pthread tools/micro/host_stream.cpp -o tools/micro/host_stream
// Run:   tools/micro/host_stream [--mb 133] [--reps 9] [--threads 1,2,4,8,16,32]
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <fstream>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace {

int cpu_node(int cpu) {
    for (int n = 0; n < 64; n++) {
        std::ifstream f("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
        if (!f) continue;
        std::string s;
        std::getline(f, s);
        size_t i = 0;
        while (i < s.size()) {
            size_t j = s.find(',', i);
            if (j == std::string::npos) j = s.size();
            const std::string r = s.substr(i, j - i);
            const size_t d = r.find('-');
            const int a = atoi(r.c_str()), b = d == std::string::npos ? a : atoi(r.c_str() + d + 1);
            if (cpu >= a && cpu <= b) return n;
            i = j + 1;
        }
    }
    return -1;
}

int llc_id(int cpu) {      // the shared_cpu_list's first CPU of the last cache level
    std::string best;
    for (int idx = 0; idx < 8; idx++) {
        std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache/index" + std::to_string(idx) +
                        "/shared_cpu_list");
        if (!f) break;
        std::getline(f, best);
    }
    return best.empty() ? cpu : atoi(best.c_str());
}

void pin(int cpu) {
    cpu_set_t s;
    CPU_ZERO(&s);
    CPU_SET(cpu, &s);
    pthread_setaffinity_np(pthread_self(), sizeof s, &s);
}

void stream_fill(uint32_t *p, size_t n, uint32_t v) {
    const __m256i x = _mm256_set1_epi32((int)v);
    for (size_t i = 0; i + 8 <= n; i += 8) _mm256_stream_si256(reinterpret_cast<__m256i *>(p + i), x);
    _mm_sfence();
}

}  // namespace

int main(int argc, char **argv) {
    size_t mb = 133;
    int reps = 9;
    std::vector<int> counts = {1, 2, 4, 8, 16, 32};
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--mb")) mb = (size_t)atol(argv[i + 1]);
        else if (!strcmp(argv[i], "--reps")) reps = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--threads")) {
            counts.clear();
            for (char *t = strtok(argv[i + 1], ","); t; t = strtok(nullptr, ",")) counts.push_back(atoi(t));
        }
    }
    // the CPUs this process may use, grouped by last-level cache
    cpu_set_t allowed;
    sched_getaffinity(0, sizeof allowed, &allowed);
    std::map<int, std::vector<int>> doms;
    for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &allowed)) doms[llc_id(c)].push_back(c);
    const int home = doms.begin()->second[0], node = cpu_node(home);
    // CPUs round-robin over the domains (one per domain first, then a second per domain, ...),
    // domains on the buffer's node first
    std::vector<int> order;
    for (size_t k = 0;; k++) {
        const size_t before = order.size();
        for (int pass = 0; pass < 2; pass++)
            for (auto &d : doms)
                if ((cpu_node(d.second[0]) == node) == (pass == 0) && k < d.second.size()) order.push_back(d.second[k]);
        if (order.size() == before) break;
    }
    const size_t bytes = mb << 20, n = bytes / 4;
    uint32_t *buf = static_cast<uint32_t *>(aligned_alloc(4096, bytes));
    {
        std::thread t([&] { pin(home); memset(buf, 0, bytes); });   // first touch: the buffer on `node`
        t.join();
    }
    printf("{\"buffer_mib\": %zu, \"buffer_node\": %d, \"domains\": %zu, \"cpus\": %d, \"results\": [", mb, node,
           doms.size(), CPU_COUNT(&allowed));
    bool first = true;
    for (int T : counts) {
        if (T > (int)order.size()) break;
        double best = 1e30;
        for (int r = 0; r < reps; r++) {
            std::atomic<int> ready{0};
            std::atomic<bool> go{false};
            std::vector<double> took(T);
            std::vector<std::thread> th;
            for (int k = 0; k < T; k++)
                th.emplace_back([&, k] {
                    pin(order[k]);
                    const size_t a = n * k / T & ~(size_t)7, b = n * (k + 1) / T & ~(size_t)7;
                    ready++;
                    while (!go.load()) {}
                    const auto t0 = std::chrono::steady_clock::now();
                    stream_fill(buf + a, b - a, 0x1E1E1Eu + r);
                    took[k] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                });
            while (ready.load() < T) {}
            const auto t0 = std::chrono::steady_clock::now();
            go = true;
            for (auto &t : th) t.join();
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        int remote = 0;
        for (int k = 0; k < T; k++) remote += cpu_node(order[k]) != node;
        printf("%s{\"threads\": %d, \"remote_threads\": %d, \"GB_per_s\": %.1f, \"ms\": %.3f}", first ? "" : ", ", T, remote,
               bytes / best / 1e9, best * 1e3);
        first = false;
        fflush(stdout);
    }
    printf("]}\n");
    free(buf);
    return 0;
}
