"""Node policy configuration.

The reference hard-codes its node policy (SURVEY §5 "Config / flag system"): 8 VFs
(dpudevicehandler.go:89), LogicalBridge / VLAN = vf + 2 (hostsidemanager.go:67,188), PF 0, two
DPU devices per NF pod (sfc.go:54-59), comm-channel port 8085 and fe80::1/::2, bridge names.
Here those values are one typed config with the reference's values as defaults, loaded from a
YAML file (SafeLoader) named by `DPU_NODE_CONFIG` or `--node-config`, overridable per field by
`DPU_CFG_<FIELD>` environment variables.  Components read `node_config()`; tests swap it with
`set_node_config()`.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field

from . import vars as V


@dataclass
class NodeConfig:
    # device plumbing
    vf_count: int = 8                  # VFs / GPU vports created at start-up
    pf: int = 0                        # host PF whose VFs back pod interfaces
    logical_bridge_offset: int = 2     # LogicalBridge (= VF VLAN) = vf + offset
    nf_devices_per_pod: int = 2        # DPU devices an NF pod requests (ingress + egress)
    resource_name: str = V.RESOURCE_NAME
    nf_nad_name: str = V.NF_NAD_NAME
    # vendor comm channel (Marvell / NetSec VSPs)
    comm_port: int = 8085
    comm_ipv6_dpu: str = "fe80::1"
    comm_ipv6_host: str = "fe80::2"
    # GPU data plane
    flow_buckets: int = 1 << 18        # 4 slots each: 1M flows at 50 % load per 2^19
    hash_mode: str = "lds"             # lds | mfma | scalar
    acl_mode: str = "mfma"             # mfma | scalar | off
    wire_port: int = 4000
    vsp_state_dir: str = ""            # journal + snapshots (checkpoint/resume); "" = off
    # live data path of the GPU VSP (vsp/gpu.py, dataplane/native_io.py)
    vport_kind: str = "veth"           # veth (kernel netdev pods, AF_PACKET rings) | xdp (veth, AF_XDP) | memif | tap
    io_queues: int = 6                 # native engine rx queues (threads), each with a ring queue per GPU
    # native engine delivery threads per queue; 0 = run to completion (each rx thread completes and
    # delivers its own bursts: one busy thread per queue).  On the GPU box (16 CPUs granted) 6 x 0
    # with 8 pod threads: 91-98 Mpps, 4 x 2: 45-59 (r6 s3 / s4, profiles/r6_s*_live_*.jsonl)
    io_workers: int = 0
    # GPU-direct egress: the ring grids write frames for memif vports into the pods' rings themselves
    # (ring.h GdeRing).  Off by default: each queue's chunks commit in ticket order over PCIe (~11
    # Mpps per queue); with run-to-completion engine threads it measured 73 vs 97 Mpps (r6 s4).
    gpu_egress: bool = False
    # the GPU node's wire port (data-plane port `wire_port`, the reference's RPM / SFP uplink):
    #   "veth"  a veth pair whose host end (`uplink_host_ifname`) the node's stack or a host bridge
    #           with the physical NIC reaches pods through (an OvS internal port's role);
    #   <name>  an existing netdev (the node's data NIC), attached through AF_PACKET rings;
    #   "memif" a shared-memory wire region (<memif dir>/wire.memif) for a user-space NIC proxy;
    #   "none"  no wire port (pods reach only each other and NF pods)
    uplink: str = "veth"
    uplink_host_ifname: str = "dpuwire"
    # daemon cadences (seconds)
    device_poll: float = 5.0           # ListAndWatch refresh (deviceplugin.go:109)
    detect_poll: float = 1.0           # platform detection (daemon.go:88)
    extra: dict = field(default_factory=dict)

    @classmethod
    def load(cls, path: str | None = None, env: dict | None = None) -> "NodeConfig":
        env = os.environ if env is None else env
        path = path or env.get("DPU_NODE_CONFIG", "")
        data: dict = {}
        if path:
            import yaml

            with open(path) as f:
                data = yaml.load(f, Loader=yaml.SafeLoader) or {}
            if not isinstance(data, dict):
                raise ValueError(f"{path}: node config must be a mapping")
        names = {f.name: f for f in dataclasses.fields(cls)}
        unknown = set(data) - set(names)
        if unknown:
            raise ValueError(f"unknown node config keys: {sorted(unknown)}")
        cfg = cls(**data)
        for name, f in names.items():
            v = env.get(f"DPU_CFG_{name.upper()}")
            if v is None or name == "extra":
                continue
            cur = getattr(cfg, name)
            setattr(cfg, name, type(cur)(v) if not isinstance(cur, bool) else v.lower() in ("1", "true", "yes"))
        cfg.validate()
        return cfg

    def validate(self) -> None:
        if not 0 <= self.vf_count <= 2048:
            raise ValueError("vf_count out of range")
        if not 1 <= self.logical_bridge_offset + max(self.vf_count - 1, 0) <= 4094:
            raise ValueError("logical bridges must stay within VLAN 1-4094")
        if self.nf_devices_per_pod < 1:
            raise ValueError("nf_devices_per_pod must be >= 1")
        if self.hash_mode not in ("lds", "mfma", "scalar") or self.acl_mode not in ("mfma", "scalar", "off"):
            raise ValueError("unknown hash / ACL mode")
        if self.vport_kind not in ("veth", "xdp", "memif", "tap"):
            raise ValueError("vport_kind is veth, xdp, memif or tap")
        if not 1 <= self.io_queues <= 64 or not 0 <= self.io_workers <= 16:
            raise ValueError("io_queues in [1, 64], io_workers in [0, 16] (0: the rx threads deliver)")
        if not self.uplink or len(self.uplink) > 15 or not 1 <= len(self.uplink_host_ifname) <= 14:
            raise ValueError("uplink is 'veth', 'none' or a netdev name; uplink_host_ifname at most 14 characters")

    def logical_bridge(self, vf: int) -> int:
        return vf + self.logical_bridge_offset


_CURRENT: NodeConfig | None = None


def node_config() -> NodeConfig:
    global _CURRENT
    if _CURRENT is None:
        _CURRENT = NodeConfig.load()
    return _CURRENT


def set_node_config(cfg: NodeConfig | None) -> None:
    global _CURRENT
    _CURRENT = cfg
