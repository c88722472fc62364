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
    """Periodically copy DataPlane per-port counters into the agent's interface statistics."""

    def __init__(self, agent, dataplane, period_s: float = 1.0):
        self.agent = agent
        self.dp = dataplane
        self.period = period_s
        self._stop = threading.Event()
        self._t: threading.Thread | None = None

    def sync_once(self) -> int:
        ctr = self.dp.port_counters()
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
