#!/bin/bash
# the GPU box's CPU resources as this process sees them
echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
grep -c ^processor /proc/cpuinfo; grep -m1 "model name" /proc/cpuinfo; grep -m1 -o -w "avx512f\|avx2" /proc/cpuinfo | sort -u
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
lscpu | grep -E "^(Thread|Core|Socket|NUMA node\(s\)|NUMA node0)" ; cat /proc/sys/kernel/unprivileged_userns_clone 2>/dev/null; unshare -U true; echo "unshare rc $?"
