"""GPU VSP: the Vendor Specific Plugin whose data plane is the MI355X pipeline.

It implements the same four services as the reference's VSPs, but instead of programming OvS
(marvell/main.go:347-563, ovs-dp/ovsdp.go:113-162) or P4 tables through p4rt-ctl
(vendor/.../ipuplugin/bridgeport.go, p4rtclient.go) it writes rows of the GPU tables
(dataplane/tables.py) and commits them to HBM between batches:

* SetNumVfs(n)            -> n vports (netdevs handed to pods by the device plugin + CNI)
* CreateBridgePort(hostP-V, mac, [vlan]) -> VF port: VLAN isolation (vid = logical bridge),
                             spoof-check on the pod MAC, egress tagging, (bridge, MAC) entry
* CreateNetworkFunction(in_mac, out_mac) -> NF steering, OvS-equivalent:
      VF  -> NF-in                      (K11  in_port=vf,actions=output:nf_in)
      NF-in, dst=VF MAC -> VF           (K12  in_port=nf_in,dl_dst=M,actions=output:vf)
      NF-out, dst=VF MAC -> NF-out      (K13  hairpin, in_port action)
      NF-out -> wire, wire -> NF-out    (K11 both ways)
* gpu-nf:// chains from the SFC reconciler -> chain-table entries (NFs run inside the kernel)

Ports: vport i = data-plane port i; the uplink ("wire", the RPM/SFP port of the reference's VSPs)
is port 4000.  All mutations happen under the VSP lock and are committed atomically per RPC.
Without an NF, VFs and the wire form one L2 bridge: known pod MACs are forwarded directly,
broadcast / unknown unicast is flooded (wire first, then the other VFs), like OvS NORMAL on the
reference's br-mrv0.

Live mode (`live=True`, `vsp --live`, what the MI355X detector deploys): pod traffic flows
through the data plane.  Vport kinds:
  * veth (default): a veth pair per vport; the pod end (`dpuvpN`, the device ID the device plugin
    hands out) is moved into the pod by the CNI (networkfn.cmd_add), the data-plane end (`dpuvpNd`)
    is read / written by the native I/O engine through AF_PACKET TPACKET_V2 rings;
  * memif: a shared-memory region per vport (<PathManager.memif_dir>/dpuvpN.memif) that the device
    plugin mounts into the pod (a DPDK-memif-style application attaches to it, no syscalls);
  * tap: a TAP netdev whose fd the VSP keeps (the CNI moves the netdev; one syscall per frame).
The native engine (dataplane/native_io.py, `live_engine="native"`) moves the frames between the
vports and every GPU's resident ring kernel; "batch" / "ring" are the Python LivePath loops.  A live vport is the pod-facing side of the VF, where
the port VLAN is already stripped: VF ports are then programmed without VLAN isolation / egress
tagging (spoof-check stays).

Checkpoint / resume (the reference's VSPs lose all state on restart): with `state_dir`
every successful mutating RPC is appended to a write-ahead journal (utils/journal.py) before the
RPC returns; `checkpoint()` writes a JSON state snapshot plus a data-plane snapshot (flows,
counters; dataplane/snapshot.py) and truncates the journal.  A new GpuVsp on the same directory
restores snapshot -> data plane -> journal tail, so vport MACs, bridge ports, NF steering, GPU
chains and installed flows survive a crash of the VSP process.
"""
from __future__ import annotations

import logging
import os
import re
import socket

import numpy as np

from ..cni.netlink import FakeNetlink, Link, NetlinkManager
from ..dataplane import tables as T
from ..dataplane.engine import DataPlane
from ..config import node_config
from ..utils.journal import Journal
from .base import VspBase

log = logging.getLogger("dpu.vsp.gpu")

WIRE_PORT = 4000
VF_BRIDGE = 1
STEER_BRIDGE = 2      # no MAC entries: every frame takes its port's default output
NF_BRIDGE_BASE = 100

# journaled RPC -> hook; args are JSON-encoded (bytes as {"hex": ...})
_MUTATING = {"SetNumVfs": "set_num_vfs", "CreateBridgePort": "create_bridge_port",
             "DeleteBridgePort": "delete_bridge_port", "CreateNetworkFunction": "create_network_function",
             "DeleteNetworkFunction": "delete_network_function", "Init": "init", "GpuChain": "on_gpu_chain",
             "InstallFlows": "_install_flows_rec"}
# installs up to this many flows are journaled record-by-record; bigger bulk loads checkpoint
JOURNAL_FLOWS_MAX = 4096


def _enc(a):
    if isinstance(a, (bytes, bytearray)):
        return {"hex": bytes(a).hex()}
    if isinstance(a, (list, tuple)):
        return [_enc(x) for x in a]
    return a


def _dec(a):
    if isinstance(a, dict) and set(a) == {"hex"}:
        return bytes.fromhex(a["hex"])
    if isinstance(a, list):
        return [_dec(x) for x in a]
    return a


def _mac_str(b: bytes) -> str:
    return ":".join(f"{x:02x}" for x in b)


def _local_mac(i: int, salt: int) -> str:
    return "02:%02x:%02x:%02x:%02x:%02x" % (0xD0 | (salt & 0xF), (i >> 16) & 0xFF, (i >> 8) & 0xFF, i & 0xFF, salt >> 4 & 0xFF)


class GpuVsp(VspBase):
    name = "amd-gpu-vsp"

    def __init__(self, path_manager=None, device: str | None = None, nl: NetlinkManager | None = None,
                 opi_port: int = 0, flow_buckets: int = 1 << 16, vport_prefix: str = "dpuvp",
                 hash_mode: str = "mfma", acl_mode: str = "mfma", state_dir: str | None = None,
                 live: bool = False, uplink=None, live_engine: str = "batch", gpus=1, vport_kind: str = "tap",
                 memif_dir: str | None = None, tx_workers: int = 1, io_queues: int = 1, placement: str = "flow"):
        super().__init__(path_manager)
        if device is None:
            try:
                import torch

                device = "cuda" if torch.cuda.is_available() else "cpu"
            except Exception:  # noqa: BLE001
                device = "cpu"
        self.device = device
        # the node's GPUs behind this VSP: 1 (self.device), N, or "all" visible MI355X (dataplane/multi.py:
        # small tables replicated, flows sharded by RSS owner, one native I/O engine steering to them)
        from ..dataplane.multi import visible_devices

        if gpus == "all":
            gpus = len(visible_devices()) if device != "cpu" else 1
        self.gpus = max(1, int(gpus))
        if placement not in ("flow", "port"):
            raise ValueError("placement is 'flow' (flows sharded) or 'port' (each vport on one GPU: hop pipeline)")
        self.placement = placement
        if vport_kind not in ("tap", "veth", "xdp", "memif"):
            raise ValueError("vport_kind is 'tap' / 'veth' / 'xdp' (netdevs; xdp: veth served through AF_XDP) "
                             "or 'memif' (shared-memory vport)")
        self.vport_kind = vport_kind
        self.memif_dir = memif_dir or (self.pm.memif_dir() if self.pm is not None else None)
        self.tx_workers = int(tx_workers)
        self.io_queues = int(io_queues)
        self.nl = nl or FakeNetlink()
        self.opi_port = opi_port
        self.flow_buckets = flow_buckets
        self.prefix = vport_prefix
        self.hash_mode, self.acl_mode = hash_mode, acl_mode
        self.dp: DataPlane | None = None
        self.vports: dict[int, dict] = {}          # idx -> {name, mac, role, vlan, pod_mac}
        self.bridge_ports: dict[str, int] = {}     # "hostP-V" -> vport idx
        self.nfs: list[dict] = []                  # {in, out, in_mac, out_mac}
        self.gpu_chains: dict[str, int] = {}
        self.dpu_mode = True
        self.healthy = True
        self._salt = int.from_bytes(os.urandom(1), "little")
        self.chain_kinds: dict[str, list[str]] = {}
        self.live = live
        if live_engine not in ("batch", "ring", "native"):
            raise ValueError("live_engine is 'batch', 'ring' or 'native'")
        if (self.gpus > 1 or vport_kind in ("memif", "veth", "xdp")) and live:
            live_engine = "native"                  # the C++ engine: RSS steering / memif / AF_PACKET vports
        self.live_engine = live_engine              # "batch" (fused kernel per cycle), "ring" (resident
                                                    # kernel) or "native" (C++ I/O engine, iox.cpp)
        self.taps: dict[int, object] = {}       # live mode: port -> TapPort
        self.livepath = None
        # live mode: the wire port (WIRE_PORT).  A vport spec (netio.TapPort, native_io.PacketVport /
        # MemifVport, anything with a packet fd), or a string resolved at Init: "veth" (a veth pair
        # whose host end, `uplink_host_ifname`, the node reaches pods through), "none", or the
        # name of an existing netdev (the node's data NIC) attached through AF_PACKET rings, or
        # "memif" (a shared-memory wire region next to the memif vports)
        self.uplink = uplink
        self._uplink_vp = None                  # the resolved wire vport (closed with the live path)
        self.port_state: dict[int, tuple[bool, bool, int]] = {}  # port -> (link, rx, mtu) from the agent
        self.agent_bridge = None
        self.journal = Journal(state_dir, "gpu-vsp") if state_dir else None
        self._replaying = False
        self.restored = 0
        if self.journal is not None:
            self._restore()

    # ------------------------------------------------------------------ helpers
    def _ensure_dp(self) -> DataPlane:
        if self.dp is None:
            kw = dict(flow_buckets=self.flow_buckets, hash_mode=self.hash_mode, acl_mode=self.acl_mode)
            if self.gpus > 1:
                from ..dataplane.multi import MultiDataPlane, visible_devices

                devs = visible_devices() if self.device != "cpu" else ["cpu"] * self.gpus
                if self.device != "cpu" and len(devs) < self.gpus:
                    raise RuntimeError(f"{self.gpus} GPUs requested, {len(devs)} visible")
                self.dp = MultiDataPlane(devs[: self.gpus], placement=self.placement, **kw)
            else:
                self.dp = DataPlane(device=self.device, **kw)
            self.dp.ports.set(WIRE_PORT, flags=T.PORT_VALID, bridge_id=VF_BRIDGE, mac="02:00:00:00:0f:a0")
            self._apply_port_state(WIRE_PORT)
            self.dp.commit(full=True)
        return self.dp

    def _commit(self) -> None:
        self.dp.commit()

    def _vport_by_mac(self, mac: str) -> int:
        mac = mac.lower()
        for i, v in self.vports.items():
            if v["mac"] == mac:
                return i
        # the NF pod may have been given the vport under another name: ask netlink
        raise KeyError(f"no vport with MAC {mac}")

    def _free_port(self) -> int:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    def _ensure_tap(self, name: str, mac: str) -> None:
        """Create the vport netdev unless it exists in any namespace (a restart must not
        duplicate a vport that the CNI already moved into a pod)."""
        if isinstance(self.nl, FakeNetlink) and not any(name in links for links in self.nl.ns.values()):
            self.nl.add_link(Link(name=name, mac=mac, up=True, kind="tap"))

    def _vf_ports(self) -> list[int]:
        return sorted(self.bridge_ports.values())

    def _program_port(self, i: int) -> None:
        v = self.vports[i]
        dp = self.dp
        if v["role"] == "vf":
            vlan_flags = 0 if self.live else T.PORT_VLAN_ISOLATE | T.PORT_TAG_EGRESS
            dp.ports.set(i, flags=T.PORT_VALID | T.PORT_SPOOFCHK | vlan_flags,
                         vlan=v["vlan"], bridge_id=VF_BRIDGE, mac=v["pod_mac"], peer_mac=v["pod_mac"],
                         default_out=WIRE_PORT)
        elif v["role"] in ("nf_in", "nf_out"):
            dp.ports.set(i, flags=T.PORT_VALID, bridge_id=v["bridge"], mac=v["mac"], peer_mac=v["mac"])
        else:
            dp.ports.set(i, flags=T.PORT_VALID, bridge_id=VF_BRIDGE, mac=v["mac"], peer_mac=v["mac"],
                         default_out=WIRE_PORT)
        self._apply_port_state(i)

    def _apply_port_state(self, i: int) -> None:
        st = self.port_state.get(i)
        if st is None or self.dp is None:
            return
        link, rx, mtu = st
        self.dp.ports.set_link(i, link)
        self.dp.ports.set_rx(i, rx)
        self.dp.ports.set_mtu(i, mtu)

    # ------------------------------------------------------------------ node agent
    def set_port_state(self, port: int, link: bool, rx: bool, mtu: int) -> None:
        """ctrl-net interface state of the function backed by `port` (cpagent.PortStateSync):
        kept across re-programming of the port, applied to the GPU port table now if it exists."""
        with self._lock:
            self.port_state[port] = (bool(link), bool(rx), int(mtu))
            if self.dp is not None and (port in self.vports or port == WIRE_PORT):
                self._apply_port_state(port)
                # running rings take it through their control mailbox (no commit); else commit
                ctrl = getattr(self.dp, "ctrl_ports", None)
                if ctrl is None or not ctrl([port]):
                    self._commit()

    def attach_agent(self, agent, state_period_s: float = 0.05, stats_period_s: float = 1.0):
        """Close the loops with the node agent: interface state -> GPU port flags, port
        counters -> the agent's interface statistics (cpagent.AgentBridge)."""
        from ..cpagent import AgentBridge

        self.agent_bridge = AgentBridge(agent, self, lambda: self.dp, state_period_s, stats_period_s).start()
        return self.agent_bridge

    def stop(self) -> None:
        if self.agent_bridge is not None:
            self.agent_bridge.stop()
            self.agent_bridge = None
        self.stop_live()
        super().stop()

    def _apply_steering(self) -> None:
        """Recompute port programming + the (bridge, MAC) table from scratch (idempotent).

        Without an NF, VFs and the wire share bridge 1 (plain L2 between pods, unknown dst -> wire).
        With NFs chained NF0..NFk, VFs and the wire move to an empty "steer" bridge so every frame
        misses the MAC table and takes its port's default output (OvS `in_port=X,actions=output:Y`):
            VF -> NF0.in,  NFi.out -> NF(i+1).in (last -> wire),  wire -> NFk.out
        and the NF-side bridges carry the return path:
            (NF0.in bridge, VF MAC) -> VF;  (NFi.in bridge, VF MAC) -> NF(i-1).out;
            (NFi.out bridge, VF MAC) -> NFi.out   (hairpin: pod-to-pod goes back through the NF)
        """
        dp = self.dp
        for i in self.vports:
            self._program_port(i)
        dp.macs.clear()
        vfs = self._vf_ports()
        dp.ports.update(WIRE_PORT, default_out=None, bridge_id=VF_BRIDGE)
        # learning only on the plain bridge: a MAC learned on the steer bridge would let a VF's
        # frame to that host bypass the NF chain
        learn = self._wire_learns() and not self.nfs
        dp.ports.a[WIRE_PORT]["flags"] = (dp.ports.a[WIRE_PORT]["flags"] & ~np.uint32(T.PORT_LEARN)) | \
            np.uint32(T.PORT_LEARN if learn else 0)
        dp.ports.version += 1
        dp.flood.set_members(VF_BRIDGE, [])
        if not self.nfs:
            # one L2 bridge: pod MACs forwarded, broadcast / unknown unicast flooded (wire first)
            for i in vfs:
                dp.macs.insert(VF_BRIDGE, self.vports[i]["pod_mac"], i)
                dp.ports.update(i, default_out=None)
            dp.flood.set_members(VF_BRIDGE, [WIRE_PORT] + vfs)   # chained rows: every VF
        else:
            for i in vfs:
                dp.ports.update(i, default_out=self.nfs[0]["in"], bridge_id=STEER_BRIDGE)
            for k, nfk in enumerate(self.nfs):
                nxt = self.nfs[k + 1]["in"] if k + 1 < len(self.nfs) else WIRE_PORT
                dp.ports.update(nfk["out"], default_out=nxt)
                for i in vfs:
                    m = self.vports[i]["pod_mac"]
                    back = i if k == 0 else self.nfs[k - 1]["out"]
                    dp.macs.insert(self.vports[nfk["in"]]["bridge"], m, back)          # K12
                    dp.macs.insert(self.vports[nfk["out"]]["bridge"], m, nfk["out"])  # K13 hairpin
            dp.ports.update(WIRE_PORT, default_out=self.nfs[-1]["out"], bridge_id=STEER_BRIDGE)
        self._commit()

    # ------------------------------------------------------------------ VSP hooks
    def _wire_vport(self):
        """The wire port's vport (live mode), resolved once from `uplink`."""
        if self._uplink_vp is not None or self.uplink is None:
            return self._uplink_vp
        up = self.uplink
        if not isinstance(up, str):
            self._uplink_vp = up
        elif up in ("", "none"):
            return None
        elif up == "memif":
            # a shared-memory wire: the external side (a DPDK-memif NIC proxy, a test) attaches to
            # <memif_dir>/wire.memif
            from ..dataplane.native_io import MemifVport, memif_dir

            d = self.memif_dir or memif_dir()
            os.makedirs(d, exist_ok=True)
            self._uplink_vp = MemifVport(os.path.join(d, "wire.memif"), ring_size=4096)
        elif up == "veth":
            from ..dataplane.native_io import PacketVport

            host = node_config().uplink_host_ifname
            try:
                self.nl.link_del(host)          # a previous VSP's pair (its engine is gone)
            except Exception:  # noqa: BLE001 - none left over
                pass
            self._uplink_vp = PacketVport.create_veth(self.nl, host)
        else:
            from ..dataplane.native_io import PacketVport

            self._uplink_vp = PacketVport.attach(up)
        return self._uplink_vp

    def _wire_learns(self) -> bool:
        """A live wire port learns the external hosts' MACs (OvS NORMAL on the reference's
        br-mrv0 / br-secondary), so pod -> external unicast is forwarded, not flooded."""
        return bool(self.live and self.uplink not in (None, "", "none"))

    def init(self, dpu_mode: bool, dpu_identifier: str):
        self.dpu_mode = dpu_mode
        self._ensure_dp()
        if self.live and self.livepath is None:
            ports = dict(self.taps)
            wire = self._wire_vport()
            if wire is not None:
                ports[WIRE_PORT] = wire
            if self.live_engine == "native":
                from ..dataplane.native_io import NativeLivePath

                planes = self.dp.planes if hasattr(self.dp, "planes") else [self.dp]
                # lane groups: every GPU brings io_queues rx threads (+ their tx workers) of its
                # own, pinned to its NUMA-local CPUs, so I/O capacity grows with the GPU count;
                # gpu_egress (node config): the grids write frames for memif vports into the pods' rings
                self.livepath = NativeLivePath(planes, ports, tx_workers=self.tx_workers, queues=self.io_queues,
                                               lane_groups=True, pin_cpus=True,
                                               gpu_egress=node_config().gpu_egress).start()
            else:
                from ..dataplane.netio import LivePath

                self.livepath = LivePath(self.dp, ports, engine=self.live_engine if self.dp.gpu else "batch").start()
        if not self.opi_port:
            self.opi_port = self._free_port()
        return "127.0.0.1", self.opi_port

    def set_num_vfs(self, n: int) -> int:
        self._ensure_dp()
        if n < 0 or n > 2048:
            raise ValueError("vport count out of range")
        for i in range(n):
            if i in self.vports:
                continue
            name, mac = f"{self.prefix}{i}", _local_mac(i, self._salt)
            if self.live and self.vport_kind == "memif":
                from ..dataplane.native_io import MemifVport, memif_dir

                d = self.memif_dir or memif_dir()
                os.makedirs(d, exist_ok=True)
                vp = MemifVport(os.path.join(d, f"{name}.memif"))
                self.taps[i] = vp
                if self.livepath is not None:
                    self.livepath.add_port(i, vp)
            elif self.live and self.vport_kind in ("veth", "xdp"):
                from ..dataplane.native_io import PacketVport, XdpVport

                vp = (XdpVport if self.vport_kind == "xdp" else PacketVport).create_veth(self.nl, name, mac)
                self.taps[i] = vp
                if self.livepath is not None:
                    self.livepath.add_port(i, vp)
            elif self.live:
                from ..dataplane.netio import TapPort

                tap = TapPort(name, mac, self.nl)
                self.nl.link_set_up(name)
                self.taps[i] = tap
                if self.livepath is not None:
                    self.livepath.add_port(i, tap)
            else:
                self._ensure_tap(name, mac)
            self.vports[i] = {"name": name, "mac": mac, "role": "free", "vlan": 0, "pod_mac": mac, "bridge": VF_BRIDGE}
            self._program_port(i)
        for i in [i for i in self.vports if i >= n and self.vports[i]["role"] == "free"]:
            self.dp.ports.clear(i)
            del self.vports[i]
            tap = self.taps.pop(i, None)
            if tap is not None:
                if self.livepath is not None:
                    self.livepath.remove_port(i)
                if hasattr(tap, "close"):
                    tap.close()
        self._commit()
        return n

    def data_path_healthy(self) -> bool:
        """The VSP and its live packet path: a failed / restarting path makes every vport
        unhealthy, so the device plugin stops handing them out (ListAndWatch)."""
        lp = self.livepath
        return self.healthy and (lp is None or bool(getattr(lp, "healthy", True)))

    def get_devices(self) -> dict[str, str]:
        h = "Healthy" if self.data_path_healthy() else "Unhealthy"
        return {v["name"]: h for v in self.vports.values()}

    def vport_path(self, idx: int) -> str | None:
        """Shared-memory vports: the region a pod attaches to (mounted into the pod by the device
        plugin, DevicePluginServer.Allocate, the way vhost-user and memif sockets are)."""
        v = self.taps.get(idx)
        return getattr(v, "path", None) if self.vport_kind == "memif" else None

    def create_bridge_port(self, name, mac, ptype, logical_bridges):
        m = re.fullmatch(r"host(\d+)-(\d+)", name)
        if not m:
            raise ValueError(f"bridge port name {name!r} is not host<pf>-<vf>")
        vf = int(m.group(2))
        if vf not in self.vports:
            raise ValueError(f"VF {vf} does not exist (SetNumVfs first)")
        vlan = int(logical_bridges[0]) if logical_bridges else node_config().logical_bridge(vf)
        if not 1 <= vlan <= 4094:
            raise ValueError(f"logical bridge / vlan {vlan} out of range 1-4094")
        v = self.vports[vf]
        v.update(role="vf", vlan=vlan, pod_mac=_mac_str(mac) if mac else v["mac"])
        self.bridge_ports[name] = vf
        self._apply_steering()

    def delete_bridge_port(self, name):
        vf = self.bridge_ports.pop(name, None)
        if vf is None:
            return
        v = self.vports[vf]
        v.update(role="free", vlan=0, pod_mac=v["mac"])
        self._apply_steering()

    def create_network_function(self, inp: str, out: str):
        i_in, i_out = self._vport_by_mac(inp), self._vport_by_mac(out)
        k = len(self.nfs)
        self.vports[i_in].update(role="nf_in", bridge=NF_BRIDGE_BASE + 2 * k)
        self.vports[i_out].update(role="nf_out", bridge=NF_BRIDGE_BASE + 2 * k + 1)
        self.nfs.append({"in": i_in, "out": i_out, "in_mac": inp.lower(), "out_mac": out.lower()})
        self._apply_steering()

    def delete_network_function(self, inp: str, out: str):
        keep = []
        for nf in self.nfs:
            if nf["in_mac"] == inp.lower() and nf["out_mac"] == out.lower():
                for i in (nf["in"], nf["out"]):
                    self.vports[i].update(role="free", bridge=VF_BRIDGE)
            else:
                keep.append(nf)
        self.nfs = keep
        self._apply_steering()

    def stop_live(self) -> None:
        if self.livepath is not None:
            self.livepath.stop()
            self.livepath = None
        for tap in self.taps.values():
            if hasattr(tap, "close"):
                tap.close()
        self.taps.clear()
        if self._uplink_vp is not None and isinstance(self.uplink, str) and hasattr(self._uplink_vp, "close"):
            self._uplink_vp.close()             # (a spec the caller gave stays the caller's)
        self._uplink_vp = None

    def on_gpu_chain(self, sfc_name: str, kinds: list[str]) -> int:
        """A gpu-nf:// chain as a chain-table entry.  A hop may name the GPU it runs on
        (``gpu-nf://acl,nat`` then ``gpu-nf://ttl@1,l2fwd@1``): the chain then hands its frames to
        that GPU's data plane mid-chain (the SFC hop pipeline across GPUs, dataplane/tables.py
        expand_hops, parallel/hops.py); the plane must exist on this node."""
        with self._lock:
            self._ensure_dp()
            planes = len(getattr(self.dp, "planes", [self.dp]))
            for k in kinds:
                at = str(k).partition("@")[2]
                if at and not 0 <= int(at) < planes:
                    raise ValueError(f"gpu-nf hop {k!r}: this node's data plane has {planes} GPU(s)")
            if sfc_name in self.gpu_chains:
                cid = self.gpu_chains[sfc_name]
                self.dp.chains.set(cid, kinds)
            else:
                cid = self.dp.chains.add(kinds)
                self.gpu_chains[sfc_name] = cid
            self.chain_kinds[sfc_name] = list(kinds)
            self._commit()
            self._journal("GpuChain", (sfc_name, list(kinds)))
            return cid

    # ------------------------------------------------------------------ checkpoint / resume
    def _journal(self, name: str, args: tuple) -> None:
        if self.journal is None or self._replaying or name not in _MUTATING:
            return
        self.journal.append({"rpc": name, "args": _enc(list(args))})
        if self.journal.needs_compaction():
            self.checkpoint()

    def _state(self) -> dict:
        return {"salt": self._salt, "dpu_mode": self.dpu_mode, "opi_port": self.opi_port,
                "vports": {str(i): v for i, v in self.vports.items()}, "bridge_ports": self.bridge_ports,
                "nfs": self.nfs, "gpu_chains": {k: [cid, self.chain_kinds.get(k, [])] for k, cid in self.gpu_chains.items()},
                "dp_snapshot": self.dp is not None}

    def _dp_snap_path(self, gen: int) -> str:
        return os.path.join(os.path.dirname(self.journal.log_path), f"gpu-vsp.dp.{gen}.npz")

    def checkpoint(self) -> None:
        """Snapshot control state + data-plane tables, then truncate the journal.

        The data-plane snapshot is written under a generation name (the journal sequence number)
        that the JSON snapshot names, so a crash between the two writes restores the previous
        generation consistently instead of pairing a new .npz with an old JSON state."""
        from ..dataplane import snapshot

        with self._lock:
            if self.journal is None:
                raise RuntimeError("GpuVsp was created without state_dir")
            state = self._state()
            gen = self.journal.seq
            if self.dp is not None:
                snapshot.save(self.dp, self._dp_snap_path(gen))
                state["dp_snapshot"] = os.path.basename(self._dp_snap_path(gen))
            self.journal.compact(state)
            d = os.path.dirname(self.journal.log_path)
            for f in os.listdir(d):  # older generations are unreachable now
                if f.startswith("gpu-vsp.dp.") and f.endswith(".npz") and f != state.get("dp_snapshot"):
                    os.unlink(os.path.join(d, f))

    def _restore(self) -> None:
        from ..dataplane import snapshot

        snap, recs = self.journal.load()
        if snap is None and not recs:
            self.journal.append({"rpc": "_meta", "salt": self._salt})
            return
        self._replaying = True
        try:
            with self._lock:
                if snap is not None:
                    self._salt = int(snap["salt"])
                    self.dpu_mode = bool(snap["dpu_mode"])
                    self.opi_port = self.opi_port or int(snap.get("opi_port") or 0)
                    self.vports = {int(i): v for i, v in snap["vports"].items()}
                    self.bridge_ports = {k: int(v) for k, v in snap["bridge_ports"].items()}
                    self.nfs = snap["nfs"]
                    if snap.get("dp_snapshot"):
                        dp = self._ensure_dp()
                        snapshot.load(dp, os.path.join(os.path.dirname(self.journal.log_path), snap["dp_snapshot"]))
                        for name, (cid, kinds) in snap["gpu_chains"].items():
                            self.gpu_chains[name] = int(cid)
                            self.chain_kinds[name] = list(kinds)
                    for v in self.vports.values():
                        self._ensure_tap(v["name"], v["mac"])
                for r in recs:
                    if r["rpc"] == "_meta":
                        self._salt = int(r["salt"])
                        continue
                    getattr(self, _MUTATING[r["rpc"]])(*_dec(r["args"]))
                    self.restored += 1
        finally:
            self._replaying = False

    # ------------------------------------------------------------------ data path access
    def install_flows(self, keys: np.ndarray, actions: np.ndarray) -> None:
        """Install exact-match flows.  Durable with `state_dir`: small installs are journaled,
        bulk loads (> JOURNAL_FLOWS_MAX) take a checkpoint before returning."""
        keys = np.ascontiguousarray(keys, np.uint32).reshape(-1, 4)
        actions = np.ascontiguousarray(actions, np.uint32).reshape(-1, 4)
        with self._lock:
            self._ensure_dp()
            self.dp.flows.insert_many(keys, actions)
            self._commit()
            if self.journal is None or self._replaying:
                return
            if len(keys) <= JOURNAL_FLOWS_MAX:
                self._journal("InstallFlows", (keys.tobytes(), actions.tobytes()))
            else:
                self.checkpoint()

    def _install_flows_rec(self, keys: bytes, actions: bytes) -> None:
        self.install_flows(np.frombuffer(keys, np.uint32).reshape(-1, 4),
                           np.frombuffer(actions, np.uint32).reshape(-1, 4))

    def process(self, frames: np.ndarray, in_ports) -> tuple[np.ndarray, np.ndarray]:
        """Run a batch through the data plane: frames [n,64] uint8, in_ports [n] -> (out, meta)."""
        from ..ops.packets import inmeta as mk_inmeta

        with self._lock:
            self._ensure_dp()
            lens = np.array([self._frame_len(f) for f in frames], np.uint32)
            im = mk_inmeta(np.asarray(in_ports), lens)
            if hasattr(self.dp, "planes"):      # several GPUs: split by owner, host arrays back
                r = self.dp.run(np.ascontiguousarray(frames), im)
                return r.out, r.meta
            if self.dp.gpu:
                import torch

                r = self.dp.run(torch.from_numpy(np.ascontiguousarray(frames)).to(self.dp.tdev),
                                torch.from_numpy(im.view(np.int32)).to(self.dp.tdev))
                torch.cuda.synchronize()
                return r.out.cpu().numpy(), r.meta.cpu().numpy().view(np.uint32)
            r = self.dp.run(np.ascontiguousarray(frames), im)
            return r.out, r.meta

    @staticmethod
    def _frame_len(f: np.ndarray) -> int:
        et = (int(f[12]) << 8) | int(f[13])
        off = 18 if et == 0x8100 else 14
        et2 = (int(f[off - 2]) << 8) | int(f[off - 1])
        if et2 == 0x0800:
            return min(64, off + ((int(f[off + 2]) << 8) | int(f[off + 3])))
        return 60 if et != 0x8100 else 64
