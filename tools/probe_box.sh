# Box facts that size the CPU side of serving: CPU quota vs affinity mask, SMT/NUMA layout, and
# which NUMA node each GPU hangs off.
mkdir -p gpurun_out
{
echo "nproc=$(nproc)"; python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)),'cpu_count',os.cpu_count())"
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/memory.max; do echo "$f: $(cat $f 2>&1)"; done
lscpu | grep -i -E "numa|socket|thread"
for c in 0 1 64 127 128 255; do echo "cpu$c pkg=$(cat /sys/devices/system/cpu/cpu$c/topology/physical_package_id) core=$(cat /sys/devices/system/cpu/cpu$c/topology/core_id) sib=$(cat /sys/devices/system/cpu/cpu$c/topology/thread_siblings_list)"; done
for d in /sys/class/drm/card*/device; do echo "$d numa=$(cat $d/numa_node 2>/dev/null) $(grep PCI_SLOT_NAME $d/uevent 2>/dev/null)"; done
for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "$n $(grep -E 'location_id|domain|gfx_target' $n/properties | tr '\n' ' ')"; done
timeout -k 5 60 python3 -c "
import torch
p=torch.cuda.get_device_properties(0)
print({k:getattr(p,k) for k in dir(p) if not k.startswith('_') and 'uuid' not in k})
"
} > gpurun_out/probe.txt 2>&1
cat gpurun_out/probe.txt
