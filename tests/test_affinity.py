"""CPU placement helpers (mlapi_amd.utils.affinity, utils.threads.effective_cpus) on fake sysfs /
cgroup trees shaped like the MI355X hosts: 2 sockets x 4 cores x 2 SMT threads, CPU N and N+8
siblings, node 0 = 0-3,8-11, node 1 = 4-7,12-15."""
import os

from mlapi_amd.utils.affinity import core_order, cpu_slices, parse_cpulist, rank_cpus
from mlapi_amd.utils.threads import cgroup_cpu_quota, effective_cpus


def _fake_host(tmp_path):
    sysfs = tmp_path / "cpu"
    for c in range(16):
        d = sysfs / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        phys = c % 8
        (d / "physical_package_id").write_text(str(phys // 4))
        (d / "core_id").write_text(str(phys % 4))
    node = tmp_path / "node"
    (node / "node0").mkdir(parents=True)
    (node / "node1").mkdir(parents=True)
    (node / "node0" / "cpulist").write_text("0-3,8-11\n")
    (node / "node1" / "cpulist").write_text("4-7,12-15\n")
    return str(sysfs), str(node)


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


def test_core_order_puts_smt_siblings_last(tmp_path):
    sysfs, _ = _fake_host(tmp_path)
    assert core_order(list(range(16)), sysfs) == [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15]
    # sibling numbering interleaved differently still yields one thread per core first
    assert core_order([8, 0, 9, 1], sysfs) == [0, 1, 8, 9]


def test_cpu_slices_budget_uses_physical_cores(tmp_path):
    sysfs, _ = _fake_host(tmp_path)
    # quota of 8 cores on a 16-thread host: 4 ranks x 2 CPUs, no two on one physical core
    sl = cpu_slices(4, list(range(16)), budget=8, sysfs=sysfs)
    assert sl == [[0, 1], [2, 3], [4, 5], [6, 7]]
    flat = [c for s in sl for c in s]
    assert len({c % 8 for c in flat}) == len(flat)
    # no budget: each rank owns whole cores (both SMT threads), never half of a core
    assert cpu_slices(2, list(range(16)), sysfs=sysfs) == [[0, 1, 2, 3, 8, 9, 10, 11], [4, 5, 6, 7, 12, 13, 14, 15]]


def test_rank_cpus_follow_gpu_numa_node(tmp_path):
    sysfs, sysnode = _fake_host(tmp_path)
    # 4 ranks, GPUs 0,1 on node 1 and GPUs 2,3 on node 0 (deliberately not rank order), budget 8
    nodes = [1, 1, 0, 0]
    got = [rank_cpus(r, 4, nodes, cpus=list(range(16)), budget=8, sysfs=sysfs, sysnode=sysnode) for r in range(4)]
    assert got == [[4, 5], [6, 7], [0, 1], [2, 3]]
    # unknown node -> plain physical-core slices
    assert rank_cpus(1, 4, None, cpus=list(range(16)), budget=8, sysfs=sysfs, sysnode=sysnode) == [2, 3]
    # node too small for its ranks (all 4 GPUs on node 0 with 4 CPUs each) -> global slices
    got = rank_cpus(3, 4, [0, 0, 0, 0], cpus=list(range(16)), budget=16, sysfs=sysfs, sysnode=sysnode)
    assert got == [6, 7, 14, 15]


def test_cgroup_quota(tmp_path):
    v2 = tmp_path / "v2"
    v2.mkdir()
    (v2 / "cpu.max").write_text("1600000 100000\n")
    assert cgroup_cpu_quota(str(v2)) == 16.0
    assert effective_cpus(str(v2)) == min(16, len(os.sched_getaffinity(0)))
    (v2 / "cpu.max").write_text("max 100000\n")
    assert cgroup_cpu_quota(str(v2)) is None
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("200000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert cgroup_cpu_quota(str(v1)) == 2.0
    assert effective_cpus(str(v1)) == min(2, len(os.sched_getaffinity(0)))
    assert cgroup_cpu_quota(str(tmp_path / "none")) is None


def _fake_mi355x_node(tmp_path, gpu_nodes=(0, 0, 0, 0, 1, 1, 1, 1)):
    """8 GPUs in KFD topology (after 2 CPU nodes), their PCI numa_node files, and 2 NUMA nodes of
    128 CPUs each (node 0 = 0-63,128-191, node 1 = 64-127,192-255) - the MI355X host layout."""
    kfd = tmp_path / "kfd"
    pci = tmp_path / "pci"
    node = tmp_path / "node"
    for n in range(2):  # CPU agents first, as KFD lists them
        (kfd / str(n)).mkdir(parents=True)
        (kfd / str(n) / "properties").write_text("cpu_cores_count 128\nsimd_count 0\nlocation_id 0\ndomain 0\n")
    for g, nn in enumerate(gpu_nodes):
        bus = 0x05 + 0x10 * g
        (kfd / str(2 + g)).mkdir(parents=True)
        (kfd / str(2 + g) / "properties").write_text(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        d = pci / f"0000:{bus:02x}:00.0"
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{nn}\n")
    (node / "node0").mkdir(parents=True)
    (node / "node1").mkdir(parents=True)
    (node / "node0" / "cpulist").write_text("0-63,128-191\n")
    (node / "node1" / "cpulist").write_text("64-127,192-255\n")
    return str(kfd), str(pci), str(node)


def test_launcher_numa_placement_is_the_gpus_node_mask(tmp_path, monkeypatch):
    """at N > 1 every rank's mask is its GPU's whole NUMA node (not a core
    slice), read from sysfs without touching the GPU."""
    from mlapi_amd.launch import rank_placement
    from mlapi_amd.utils.affinity import gpu_numa_nodes, kfd_gpu_bdfs

    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    kfd, pci, node = _fake_mi355x_node(tmp_path)
    assert kfd_gpu_bdfs(kfd)[:2] == ["0000:05:00.0", "0000:15:00.0"]
    assert gpu_numa_nodes(kfd, pci) == [0, 0, 0, 0, 1, 1, 1, 1]
    masks = rank_placement("numa", 8, sys_kfd=kfd, sys_pci=pci, sysnode=node, cpus=list(range(256)))
    n0 = list(range(0, 64)) + list(range(128, 192))
    n1 = list(range(64, 128)) + list(range(192, 256))
    assert masks == [n0] * 4 + [n1] * 4
    # the mask never exceeds what the process may use
    masks = rank_placement("numa", 8, sys_kfd=kfd, sys_pci=pci, sysnode=node, cpus=list(range(0, 256, 2)))
    assert all(c % 2 == 0 for m in masks for c in m) and len(masks[0]) == 64
    # HIP_VISIBLE_DEVICES remaps ordinals: rank 0 drives physical GPU 5 (node 1)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5,1")
    assert gpu_numa_nodes(kfd, pci) == [1, 0]
    # no topology (a container without KFD sysfs): ranks stay unpinned
    assert rank_placement("numa", 2, sys_kfd=str(tmp_path / "none"), sys_pci=pci, sysnode=node) == [[], []]
    assert rank_placement("off", 3) == [[], [], []]
