"""Node control agent (native `_agent` module) — Python-side constants and glue.

The agent itself is C++ (csrc/agent: shared-memory control mailbox, ctrl-net command handler,
heartbeat/reset handling, plugin TCP relay; standalone binary `native/bin/dpu-cp-agent`).  It is
the MI355X counterpart of the reference's Marvell `octep_cp_agent` (SURVEY NAT1-NAT10): the host
netdev side talks to it over the mailbox; here it fronts the GPU data plane, so interface
statistics come from the data plane's per-port counters (`StatsBridge`).
"""
from __future__ import annotations

import enum
import threading

from .native import agent as _agent_mod


class H2F(enum.IntEnum):
    MTU = 1
    MAC = 2
    GET_IF_STATS = 3
    GET_XSTATS = 4
    GET_Q_STATS = 5
    LINK_STATUS = 6
    RX_STATE = 7
    LINK_INFO = 8
    GET_INFO = 9
    DEV_REMOVE = 10
    OFFLOADS = 11


class Reply(enum.IntEnum):
    OK = 0
    GENERIC_FAIL = 1
    INVALID_PARAM = 2
    UNSUPPORTED = 3


GET, SET = 0, 1
FLAG_REQ, FLAG_RESP, FLAG_NOTIFY, FLAG_CUSTOM = 1, 2, 4, 8


def native():
    return _agent_mod()


def default_config(n_vfs: int = 8, hb_interval_ms: int = 1000, hb_miss_count: int = 20, port_base: int = 0) -> str:
    """One PEM, one PF, `n_vfs` VFs; VF i backed by data-plane port `port_base + i`."""
    vfs = ",\n".join(
        f'{{ idx = {i}; mac_addr = [0x02, 0xD0, 0x00, 0x00, 0x{(i >> 8) & 0xFF:02x}, 0x{i & 0xFF:02x}]; '
        f"link_state = 1; rx_state = 1; autoneg = 0x3; pause_mode = 0x3; speed = 200000; "
        f"supported_modes = 0x3; advertised_modes = 0x1; dp_port = {port_base + i}; }}"
        for i in range(n_vfs))
    return f"""soc = {{
  pems = ( {{ idx = 0;
    pfs = ( {{ idx = 0; mac_addr = [0x02, 0xD0, 0x00, 0x00, 0xFF, 0xFF];
      link_state = 1; rx_state = 1; autoneg = 0x3; pause_mode = 0x3; speed = 200000;
      supported_modes = 0x3; advertised_modes = 0x1; hb_interval = {hb_interval_ms}; hb_miss_count = {hb_miss_count};
      dp_port = 4000;
      vfs = ( {vfs} ); }} ); }} );
}};
"""


class StatsBridge:
    """Periodically copy DataPlane per-port counters into the agent's interface statistics.
    `dataplane` is a DataPlane or a callable returning one (None while it does not exist yet)."""

    def __init__(self, agent, dataplane, period_s: float = 1.0):
        self.agent = agent
        self.dp = dataplane
        self.period = period_s
        self._stop = threading.Event()
        self._t: threading.Thread | None = None

    def sync_once(self) -> int:
        dp = self.dp() if callable(self.dp) else self.dp
        if dp is None:
            return 0
        ctr = dp.port_counters()
        drops = 0
        n = 0
        for pem, pf, vf in self.agent.functions():
            port = self.agent.iface(pem, pf, vf)["dp_port"]
            if port < 0 or port >= len(ctr):
                continue
            rx_p, rx_b, tx_p, tx_b = (int(x) for x in ctr[port])
            self.agent.update_stats(pem, pf, vf, rx_p, rx_b, tx_p, tx_b, drops, 0)
            n += 1
        return n

    def start(self) -> "StatsBridge":
        def run():
            while not self._stop.wait(self.period):
                self.sync_once()

        self._t = threading.Thread(target=run, daemon=True, name="agent-stats")
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=5)


class DataPlanePorts:
    """`set_port_state` target for a bare DataPlane (a VSP implements the same method itself)."""

    def __init__(self, dataplane):
        self.dp = dataplane

    def set_port_state(self, port: int, link: bool, rx: bool, mtu: int) -> None:
        p = self.dp.ports
        p.set_link(port, link)
        p.set_rx(port, rx)
        p.set_mtu(port, mtu)
        ctrl = getattr(self.dp, "ctrl_ports", None)   # running rings: their control mailbox
        if ctrl is None or not ctrl([port]):
            self.dp.commit()


class PortStateSync:
    """ctrl-net interface state -> GPU port flags (the control loop of the reference's
    octep_cp_agent loop.c:107-288, where SET_MTU / LINK_STATUS / RX_STATE / DEV_REMOVE reconfigure
    the SoC interface).  The agent bumps `state_gen` on every such change; `sync_once` re-applies
    each function's state to its data-plane port when it moved:
        link down or removed -> PORT_LINK_DOWN (the port neither receives nor sends)
        RX state off         -> PORT_RX_OFF    (nothing is delivered to the port)
        MTU                  -> port egress MTU (larger frames dropped as too_big)
    `target` has `set_port_state(port, link, rx, mtu)` (GpuVsp, or DataPlanePorts)."""

    def __init__(self, agent, target):
        self.agent = agent
        self.target = target
        self.gen = -1
        self.applied: dict[int, tuple] = {}

    def sync_once(self, force: bool = False) -> int:
        g = self.agent.state_gen
        if g == self.gen and not force:
            return 0
        self.gen = g
        n = 0
        for pem, pf, vf in self.agent.functions():
            s = self.agent.iface(pem, pf, vf)
            port = s["dp_port"]
            if port < 0:
                continue
            st = (bool(s["link"]) and not s["removed"], bool(s["rx"]) and not s["removed"], int(s["mtu"]))
            if self.applied.get(port) == st and not force:
                continue
            self.target.set_port_state(port, *st)
            self.applied[port] = st
            n += 1
        return n


class AgentBridge:
    """One thread that keeps the agent and the data plane in step: interface state -> port flags
    every `state_period_s` (cheap: one atomic read when nothing changed), port counters -> agent
    interface statistics every `stats_period_s`."""

    def __init__(self, agent, target, dataplane, state_period_s: float = 0.05, stats_period_s: float = 1.0):
        self.state = PortStateSync(agent, target)
        self.stats = StatsBridge(agent, dataplane, stats_period_s)
        self.state_period = state_period_s
        self.stats_period = stats_period_s
        self._stop = threading.Event()
        self._t: threading.Thread | None = None
        self.errors = 0

    def _run(self) -> None:
        import logging
        import time

        log = logging.getLogger("dpu.cpagent")
        next_stats = time.monotonic() + self.stats_period
        while not self._stop.wait(self.state_period):
            try:
                self.state.sync_once()
                if time.monotonic() >= next_stats:
                    next_stats += self.stats_period
                    self.stats.sync_once()
            except Exception:  # noqa: BLE001 - the loop outlives a bad sync; counted and logged
                self.errors += 1
                log.exception("agent bridge sync failed")

    def start(self) -> "AgentBridge":
        self.state.sync_once(force=True)
        self._t = threading.Thread(target=self._run, daemon=True, name="agent-bridge")
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=5)
