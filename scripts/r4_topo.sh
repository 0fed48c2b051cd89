#!/bin/bash
# host topology of the GPU box (NUMA node of the GPU, CPUs this job may use)
echo "nproc: $(nproc)"; grep -E 'Cpus_allowed_list|Mems_allowed_list' /proc/self/status
ls /sys/devices/system/node/ | grep node
for n in /sys/devices/system/node/node*; do echo "$n cpus $(cat $n/cpulist) mem $(grep MemTotal $n/meminfo | awk '{print $4 $5}')"; done
for c in /sys/class/drm/card*/device; do [ -f $c/numa_node ] && echo "$c numa $(cat $c/numa_node) $(cat $c/uevent | grep PCI_SLOT_NAME)"; done
df -h /dev/shm /tmp | cat
