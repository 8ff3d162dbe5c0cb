#include "host_cpus.h"

#include <sched.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace zpx {

namespace {
int probe_budget()
{
    int n = static_cast<int>(std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = CPU_COUNT(&set);
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char quota[32] = {};
        long period = 0;
        if (fscanf(f, "%31s %ld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
            const long q = atol(quota);
            if (q > 0) {
                const int cap = static_cast<int>(std::ceil(double(q) / double(period)));
                if (cap < n) n = cap;
            }
        }
        fclose(f);
    }
    return n > 0 ? n : 1;
}
} // namespace

int host_cpu_budget()
{
    static const int n = probe_budget();
    return n;
}

} // namespace zpx
