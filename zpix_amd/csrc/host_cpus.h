// The host CPUs this process may use, for sizing the entropy / inflate pools.
#pragma once

namespace zpx {

// The affinity set capped by a cgroup v2 CPU quota (/sys/fs/cgroup/cpu.max):
// a GPU box shares its host, so hardware_concurrency() overstates what a
// process gets (256 hardware threads against a 16-CPU quota on the bench
// boxes).  Read once; at least 1.  zpix_amd/shard.py host_cpu_budget() is
// the same rule for the Python side.
int host_cpu_budget();

} // namespace zpx
