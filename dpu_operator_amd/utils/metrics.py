"""Prometheus metrics + health probes.

The reference exposes controller-runtime metrics on :18090 and probes on :18091 (cmd/main.go:50-51,
SURVEY §5 "metrics").  Here one registry carries:
* control-plane counters (reconciles, CNI requests by command/result, VSP RPCs, device-plugin
  allocations) — `CONTROL` below, incremented by the components;
* `DataPlaneCollector`: per-port rx/tx packets+bytes, drops by reason, installed flows, entries
  per table (flows, MACs static / learned, ACL rules, routes, nexthops, ECMP / LAG / flood groups,
  tunnels, VM MAC maps), flow-table hits / misses, packet-path latency histograms — read from a
  DataPlane at scrape time (counters are 64-bit on the host, harvested from the packed device
  counters).
`MetricsServer` serves /metrics (text exposition) and `ProbeServer` /healthz + /readyz with
pluggable checks.
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily

REGISTRY = CollectorRegistry(auto_describe=True)


class _Control:
    def __init__(self, reg: CollectorRegistry):
        self.reconciles = Counter("dpu_reconcile_total", "Reconcile calls", ["controller", "result"], registry=reg)
        self.cni_requests = Counter("dpu_cni_requests_total", "CNI requests served", ["command", "result"], registry=reg)
        self.vsp_calls = Counter("dpu_vsp_calls_total", "VSP RPCs", ["method", "result"], registry=reg)
        self.allocations = Counter("dpu_device_plugin_allocations_total", "Device plugin Allocate calls", registry=reg)
        self.devices = Gauge("dpu_devices", "Devices advertised to the kubelet", ["health"], registry=reg)
        self.p4_writes = Counter("dpu_p4_writes_total", "P4 table writes", ["verb", "result"], registry=reg)
        self.batch_seconds = Histogram("dpu_dataplane_batch_seconds", "Host-observed data-plane batch time",
                                       buckets=(1e-5, 3e-5, 1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1), registry=reg)


CONTROL = _Control(REGISTRY)


class DataPlaneCollector:
    """Scrape-time export of a DataPlane's counters (no per-packet Python work).  `dataplane` is a
    DataPlane or a callable returning one (a VSP creates its data plane on Init: nothing is
    exported before that)."""

    def __init__(self, dataplane, name: str = "gpu0", max_ports: int = 4096):
        self._dp = dataplane
        self.name = name
        self.max_ports = max_ports

    @property
    def dp(self):
        return self._dp() if callable(self._dp) else self._dp

    def collect(self):
        dp = self.dp
        if dp is None:
            return
        yield from self._collect(dp)

    def _collect(self, dp):
        from ..dataplane import tables as T

        ctr = dp.port_counters()
        labels = ["dataplane", "port"]
        rx_p = CounterMetricFamily("dpu_port_rx_packets", "Packets received per port", labels=labels)
        rx_b = CounterMetricFamily("dpu_port_rx_bytes", "Bytes received per port", labels=labels)
        tx_p = CounterMetricFamily("dpu_port_tx_packets", "Packets transmitted per port", labels=labels)
        tx_b = CounterMetricFamily("dpu_port_tx_bytes", "Bytes transmitted per port", labels=labels)
        active = (ctr[:, 0] > 0) | (ctr[:, 2] > 0)
        for port in active.nonzero()[0][: self.max_ports]:
            lv = [self.name, str(int(port))]
            rx_p.add_metric(lv, float(ctr[port, 0]))
            rx_b.add_metric(lv, float(ctr[port, 1]))
            tx_p.add_metric(lv, float(ctr[port, 2]))
            tx_b.add_metric(lv, float(ctr[port, 3]))
        yield from (rx_p, rx_b, tx_p, tx_b)
        drops = CounterMetricFamily("dpu_drops", "Dropped packets by reason", labels=["dataplane", "reason"])
        for reason, n in sorted(dp.drop_counters().items()):
            drops.add_metric([self.name, reason], float(n))
        yield drops
        flows = GaugeMetricFamily("dpu_flows_installed", "Exact-match flows installed", labels=["dataplane"])
        flows.add_metric([self.name], float(len(dp.flows)))
        yield flows
        cap = GaugeMetricFamily("dpu_flow_capacity", "Flow table slots", labels=["dataplane"])
        cap.add_metric([self.name], float(dp.flows.nbuckets * 4))
        yield cap
        ports = GaugeMetricFamily("dpu_ports_valid", "Valid data-plane ports", labels=["dataplane"])
        f = dp.ports.a["flags"]
        ports.add_metric([self.name], float((f & T.PORT_VALID).astype(bool).sum()))
        yield ports
        down = GaugeMetricFamily("dpu_ports_down", "Valid ports whose link is down or RX is off",
                                 labels=["dataplane", "state"])
        valid = (f & T.PORT_VALID).astype(bool)
        down.add_metric([self.name, "link_down"], float((valid & (f & T.PORT_LINK_DOWN).astype(bool)).sum()))
        down.add_metric([self.name, "rx_off"], float((valid & (f & T.PORT_RX_OFF).astype(bool)).sum()))
        yield down
        # per-table occupancy and flow-table hit / miss (per-table hit/miss)
        ent = GaugeMetricFamily("dpu_table_entries", "Entries per data-plane table", labels=["dataplane", "table"])
        for name, n in _table_sizes(dp).items():
            ent.add_metric([self.name, name], float(n))
        yield ent
        hits = int(dp.flow_totals[:, 0].sum()) if getattr(dp, "flow_totals", None) is not None else 0
        past_ingress = int(ctr[:, 0].sum()) - sum(n for r, n in dp.drop_counters().items() if r in _INGRESS_DROPS)
        hm = CounterMetricFamily("dpu_flow_lookups", "Exact-match flow lookups past ingress checks, by result (hits "
                                 "as of the last per-flow counter harvest)", labels=["dataplane", "result"])
        hm.add_metric([self.name, "hit"], float(hits))
        hm.add_metric([self.name, "miss"], float(max(past_ingress - hits, 0)))
        yield hm
        lat = HistogramMetricFamily("dpu_packet_latency_seconds",
                                    "Packet-path latency by stage (utils/latency.py: rx, pipeline, side, tx, "
                                    "batch per live batch; device per sampled packet)", labels=["dataplane", "stage"])
        for stage, h in dp.latency.items():
            b, total = h.buckets()
            lat.add_metric([self.name, stage], b, total)
        yield lat


# drop reasons decided before the flow lookup (ingress_stage)
_INGRESS_DROPS = ("bad_port", "vlan_drop", "spoof", "malformed")


def _table_sizes(dp) -> dict:
    """Occupancy of every table the data plane holds (attributes a DataPlane may lack are skipped)."""
    from ..dataplane import tables as T

    out = {"flows": len(dp.flows), "acl_rules": len(dp.acl.rules), "chains": int(dp.chains.n)}
    v = dp.macs.a["valid"]
    out["macs_static"] = int((v == T.MAC_STATIC).sum())
    out["macs_learned"] = int((v == T.MAC_LEARNED).sum())
    for name, attr in (("routes_v4", "routes"), ("routes_v6", "routes6"), ("tunnel_terms", "terms"),
                       ("vm_mac_maps", "vmmac")):
        t = getattr(dp, attr, None)
        if t is None:
            continue
        out[name] = len(t) if hasattr(t, "__len__") else int(getattr(t, "n", 0))
    for name, attr in (("nexthops", "nexthops"), ("ecmp_groups", "ecmp"), ("lag_groups", "lag"), ("tunnels_v4", "tunnels"),
                       ("tunnels_v6", "tunnels6"), ("flood_groups", "flood")):
        t = getattr(dp, attr, None)
        if t is not None:
            out[name] = int(getattr(t, "n", 0))
    return out


def register_dataplane(dataplane, name: str = "gpu0", registry: CollectorRegistry = REGISTRY) -> DataPlaneCollector:
    c = DataPlaneCollector(dataplane, name)
    registry.register(c)
    return c


class _Srv:
    def __init__(self, address: str):
        host, _, port = address.rpartition(":")
        self.addr = (host or "0.0.0.0", int(port))
        self._srv: ThreadingHTTPServer | None = None
        self.port = 0

    def _handler(self):
        raise NotImplementedError

    def start(self):
        self._srv = ThreadingHTTPServer(self.addr, self._handler())
        self._srv.daemon_threads = True
        self.port = self._srv.server_address[1]
        threading.Thread(target=self._srv.serve_forever, daemon=True).start()
        return self

    def stop(self) -> None:
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()


class MetricsServer(_Srv):
    def __init__(self, address: str = ":18090", registry: CollectorRegistry = REGISTRY):
        super().__init__(address)
        self.registry = registry

    def _handler(self):
        reg = self.registry

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path.split("?")[0] != "/metrics":
                    self.send_response(404)
                    self.end_headers()
                    return
                body = generate_latest(reg)
                self.send_response(200)
                self.send_header("Content-Type", CONTENT_TYPE_LATEST)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        return H


class ProbeServer(_Srv):
    """/healthz and /readyz; each has a list of named check callables returning bool."""

    def __init__(self, address: str = ":18091"):
        super().__init__(address)
        self.health: dict[str, callable] = {"ping": lambda: True}
        self.ready: dict[str, callable] = {"ping": lambda: True}

    def _handler(self):
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                checks = {"/healthz": outer.health, "/readyz": outer.ready}.get(self.path)
                if checks is None:
                    self.send_response(404)
                    self.end_headers()
                    return
                failed = [n for n, fn in checks.items() if not _ok(fn)]
                body = (b"ok" if not failed else ("failed: " + ",".join(failed)).encode())
                self.send_response(200 if not failed else 500)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        return H


def _ok(fn) -> bool:
    try:
        return bool(fn())
    except Exception:  # noqa: BLE001
        return False
