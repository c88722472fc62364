"""`vsp` — run a Vendor Specific Plugin on the vendor-plugin socket.

The reference builds one binary per vendor (cmd/intelvsp/intelvsp.go, marvell/main.go:823,
intel-netsec/main.go:627, mock-vsp); here `--vendor` selects it:
  amd-gpu    GPU VSP on the MI355X data plane (vsp/gpu.py)
  mock       mock VSP (Init -> 127.0.0.1:50051, four healthy devices)
  marvell    Marvell VSP; OvS-equivalent bridge on the GPU data plane (--debug-dp: log only)
  netsec     Intel NetSec accelerator VSP on the GPU data plane
  intel-ipu  Intel IPU VSP writing P4 rules to the pipeline server (--p4rt-addr)

amd-gpu extras:
  --metrics-bind-address  serve the data plane's metrics (per-port counters, drops, flows, the
                          packet-path latency histograms) on /metrics of this address
  --agent-mbox PATH       run the node control agent (csrc/agent) on this mailbox and close its
                          loops with the data plane: ctrl-net MTU / link / RX state -> GPU port
                          table, port counters -> agent interface statistics (cpagent.AgentBridge)
"""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import threading

from ..config import NodeConfig, node_config, set_node_config
from ..utils.paths import PathManager


def build_vsp(a, pm: PathManager):
    if a.vendor == "mock":
        from ..vsp.base import MockVsp

        return MockVsp(pm)
    if a.vendor == "amd-gpu":
        from ..vsp.gpu import GpuVsp

        cfg = node_config()
        nl = None
        if a.live:
            from ..cni.netlink import RtNetlink

            nl = RtNetlink()
        return GpuVsp(pm, device=a.device or None, flow_buckets=a.flow_buckets or cfg.flow_buckets,
                      hash_mode=cfg.hash_mode, acl_mode=cfg.acl_mode,
                      state_dir=a.state_dir or cfg.vsp_state_dir or None, nl=nl, live=a.live,
                      live_engine=a.live_engine, gpus=a.gpus if a.gpus == "all" else int(a.gpus),
                      vport_kind=a.vport_kind or cfg.vport_kind, tx_workers=cfg.io_workers if a.io_workers < 0 else a.io_workers,
                      io_queues=a.io_queues or cfg.io_queues, placement=a.placement,
                      uplink=(a.uplink or cfg.uplink) if a.live else None)
    from ..cni.netlink import RtNetlink
    from ..platform.platform import SysfsPlatform
    from ..utils.cmdrunner import HostRunner

    plat, nl, runner = SysfsPlatform(a.sys_root), RtNetlink(), HostRunner()

    def dataplane():
        """One GPU, or with --gpus N|all every one behind a MultiDataPlane (tables replicated,
        flows sharded by RSS owner, the OvS flow tables compiled once for all of them)."""
        from ..dataplane.engine import DataPlane
        from ..dataplane.multi import MultiDataPlane, visible_devices

        buckets = a.flow_buckets or node_config().flow_buckets
        n = len(visible_devices()) if a.gpus == "all" else int(a.gpus)
        if n > 1:
            dp = MultiDataPlane(visible_devices()[:n], placement=a.placement, flow_buckets=buckets)
        else:
            dp = DataPlane(device=a.device or "cuda", flow_buckets=buckets)
        dp.commit(full=True)
        return dp

    def live_path(dp):
        """--live: the bridge's netdev ports (uplink, VF representors, NF ports) run on the native
        I/O engine as AF_PACKET ports, ring kernels behind it (started with no port; OvS add-port
        adds them)."""
        from ..dataplane.native_io import NativeLivePath

        cfg = node_config()
        return NativeLivePath(dp, {}, tx_workers=cfg.io_workers if a.io_workers < 0 else a.io_workers,
                              queues=a.io_queues or cfg.io_queues).start()

    if a.vendor == "marvell":
        from ..vsp import marvell as M

        ddp = M.DebugDataPlane() if a.debug_dp else M.GpuOvsDataPlane(
            dataplane(), uplink_name=a.uplink or "rpm0", live_factory=live_path if a.live else None)
        return M.MarvellVsp(plat, nl, runner, ddp, pm, a.sys_root)
    if a.vendor == "netsec":
        from ..vsp.netsec import NetsecVsp

        return NetsecVsp(plat, nl, runner, dataplane(), pm, a.sys_root)
    if a.vendor == "intel-ipu":
        from ..dataplane.p4server import GrpcP4rtClient
        from ..vsp.intel_ipu import IntelIpuVsp

        accs = [m.strip() for m in a.acc_macs.split(",") if m.strip()]
        return IntelIpuVsp(GrpcP4rtClient(a.p4rt_addr), accs, path_manager=pm, mode=a.mode)
    raise SystemExit(f"unknown vendor {a.vendor!r}")


def main(argv=None, stop: threading.Event | None = None) -> int:
    a = parse_args(argv)
    if a.node_config:
        set_node_config(NodeConfig.load(a.node_config))
    logging.basicConfig(level=logging.INFO)
    vsp = build_vsp(a, PathManager(a.root)).start()
    services = _extras(a, vsp)
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    if getattr(vsp, "journal", None) is not None:
        vsp.checkpoint()  # clean shutdown: snapshot so the next start skips the replay
    vsp.stop()
    for svc in reversed(services):
        svc.stop()
    return 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="vsp")
    ap.add_argument("--vendor", default="amd-gpu", choices=["amd-gpu", "mock", "marvell", "netsec", "intel-ipu"])
    ap.add_argument("--root", default="/")
    ap.add_argument("--sys-root", default="/")
    ap.add_argument("--device", default="")
    ap.add_argument("--flow-buckets", type=int, default=0, help="0 = node config (default 2^18)")
    ap.add_argument("--node-config", default="", help="node policy YAML (config.py); also DPU_NODE_CONFIG")
    ap.add_argument("--debug-dp", action="store_true")
    ap.add_argument("--uplink", default="",
                    help="wire port: marvell: the RPM netdev (default rpm0); amd-gpu --live: 'veth' (a host-side "
                         "veth pair), 'none' or an existing netdev (the node's data NIC); default: node config uplink")
    ap.add_argument("--p4rt-addr", default="127.0.0.1:9559")
    ap.add_argument("--acc-macs", default="")
    ap.add_argument("--mode", default="ipu")
    ap.add_argument("--state-dir", default="", help="amd-gpu: journal + snapshot directory (resume on restart)")
    ap.add_argument("--live", action="store_true",
                    help="amd-gpu: vports are real netdevs and pod traffic flows through the data plane; "
                         "marvell: the OvS bridge's netdev ports run on the native I/O engine")
    ap.add_argument("--live-engine", default="native", choices=["batch", "ring", "native"],
                    help="amd-gpu --live: fused kernel per poll cycle (Python loop), the persistent ring kernel on "
                         "pinned host slots (Python loop), or the native C++ I/O engine + ring kernel")
    ap.add_argument("--gpus", default="1", help="amd-gpu / marvell / netsec: GPUs behind the VSP (a number or 'all'): tables "
                    "replicated, flows sharded by RSS owner, the native engine steering frames to their owner")
    ap.add_argument("--placement", default="flow", choices=["flow", "port"],
                    help="--gpus > 1: frames run on their flow's GPU (flows sharded by RSS owner) or on their "
                         "ingress port's GPU (flows replicated: the SFC hop pipeline across GPUs)")
    ap.add_argument("--vport-kind", default="", choices=["", "veth", "xdp", "tap", "memif"],
                    help="amd-gpu --live: vports as veth pairs (kernel-netdev pods, AF_PACKET rings), TAP "
                         "netdevs or shared-memory (memif) regions; default: node config vport_kind (veth)")
    ap.add_argument("--io-queues", type=int, default=0,
                    help="native engine rx queues (threads), each with a ring queue on every GPU (0: node config)")
    ap.add_argument("--io-workers", type=int, default=-1,
                    help="native engine delivery threads per queue (0: run to completion, the rx threads deliver; "
                         "-1: node config)")
    ap.add_argument("--metrics-bind-address", default="", help="amd-gpu: data-plane /metrics address (off if empty)")
    ap.add_argument("--agent-mbox", default="", help="amd-gpu: run the node control agent on this mailbox path")
    ap.add_argument("--agent-config", default="", help="agent SoC config file (default: one PF + --agent-vfs VFs)")
    ap.add_argument("--agent-vfs", type=int, default=8)
    return ap.parse_args(argv)


def _extras(a, vsp) -> list:
    """Metrics server and node agent around a GPU VSP; returns what to stop at shutdown."""
    out = []
    if a.vendor != "amd-gpu":
        return out
    if a.metrics_bind_address:
        from prometheus_client import CollectorRegistry

        from ..utils.metrics import MetricsServer, register_dataplane

        reg = CollectorRegistry()
        register_dataplane(lambda: vsp.dp, "gpu0" if vsp.gpus == 1 else f"gpu0-{vsp.gpus - 1}", reg)
        vsp.metrics = MetricsServer(a.metrics_bind_address, reg).start()
        out.append(vsp.metrics)
    if a.agent_mbox:
        from .. import cpagent
        from ..native import agent as native_agent

        A = native_agent()
        cfg = open(a.agent_config).read() if a.agent_config else cpagent.default_config(n_vfs=a.agent_vfs)
        ag = A.Agent(a.agent_mbox, cfg)
        ag.start()
        vsp.agent = ag
        vsp.attach_agent(ag)
        out.append(ag)
    return out


if __name__ == "__main__":
    sys.exit(main())
