"""Pipeline server (the infrap4d role) and P4 runtime clients.

`P4rtServer` hosts one `P4Runtime` per bridge (br0 ...) over gRPC (`mi355x.p4rt.v1.P4rt`):
Write (INSERT/DELETE of p4rt-ctl entry strings), Read, SetPipe (load a P4Info text), GetPipe.
Errors are gRPC statuses whose details start with the P4Runtime code name, so the callers'
string checks (ALREADY_EXISTS / INVALID_ARGUMENT, p4rtclient.go:74-101) behave the same.

Clients:
* `GrpcP4rtClient`  — direct gRPC.
* `CliP4rtClient`   — runs the `p4rt-ctl` CLI (cmd/p4rt_ctl.py) through a Runner, like the
  reference's RunP4rtCtlCommand (utils.go:129-156, serialised by one lock).
* `program_rules()` — the reference's ProgramFXPP4Rules policy: on ALREADY_EXISTS delete the
  key and re-add; on INVALID_ARGUMENT retry once; other failures are reported (the reference
  only logs them) in the returned list.
"""
from __future__ import annotations

import logging
import threading
from concurrent import futures
from dataclasses import dataclass

import grpc

from ..proto import p4rt as pb
from ..proto.grpcutil import Stub, service_handler
from .p4info import MI355X_P4INFO, MI355X_P4INFO_TEXT, P4Info
from .p4rt import P4Error, P4Runtime

log = logging.getLogger("dpu.p4rt")

_CODES = {
    "ALREADY_EXISTS": grpc.StatusCode.ALREADY_EXISTS, "NOT_FOUND": grpc.StatusCode.NOT_FOUND,
    "INVALID_ARGUMENT": grpc.StatusCode.INVALID_ARGUMENT, "RESOURCE_EXHAUSTED": grpc.StatusCode.RESOURCE_EXHAUSTED,
    "FAILED_PRECONDITION": grpc.StatusCode.FAILED_PRECONDITION,
}


class P4rtServer:
    def __init__(self, runtimes: dict[str, P4Runtime] | None = None, p4info_text: str = MI355X_P4INFO_TEXT):
        self.runtimes = runtimes if runtimes is not None else {"br0": P4Runtime()}
        self.p4info_text = {b: p4info_text for b in self.runtimes}
        self._server: grpc.Server | None = None
        self.port = 0
        self._lock = threading.Lock()

    def _rt(self, bridge: str, context) -> P4Runtime:
        rt = self.runtimes.get(bridge or "br0")
        if rt is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"NOT_FOUND: no bridge {bridge}")
        return rt

    def Write(self, request, context):
        rt = self._rt(request.bridge, context)
        n = 0
        with self._lock:
            for u in request.updates:
                try:
                    if u.type == pb.INSERT:
                        rt.add_entry(u.table, u.entry)
                    elif u.type == pb.DELETE:
                        rt.del_entry(u.table, u.entry)
                    elif u.type == pb.MODIFY:
                        try:
                            rt.del_entry(u.table, u.entry.split(",action=")[0])
                        except P4Error:
                            pass
                        rt.add_entry(u.table, u.entry)
                    else:
                        raise P4Error("INVALID_ARGUMENT", "update type unspecified")
                except P4Error as e:
                    context.abort(_CODES.get(e.code, grpc.StatusCode.UNKNOWN), str(e))
                n += 1
        return pb.WriteResponse(applied=n)

    def Read(self, request, context):
        rt = self._rt(request.bridge, context)
        try:
            rows = rt.get_entries(request.table or None)
        except P4Error as e:
            context.abort(_CODES.get(e.code, grpc.StatusCode.UNKNOWN), str(e))
        return pb.ReadResponse(entries=[pb.TableEntry(table=e.table, entry=entry_text(rt.p4info, e)) for e in rows])

    def SetPipe(self, request, context):
        rt = self._rt(request.bridge, context)
        try:
            info = P4Info.from_text(request.p4info_text)
        except ValueError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"INVALID_ARGUMENT: {e}")
        rt.set_pipe(info)
        self.p4info_text[request.bridge or "br0"] = request.p4info_text
        names = {t.name for t in info.tables.values()}
        return pb.SetPipeResponse(tables=len(names), actions=len({a.name for a in info.actions.values()}))

    def GetPipe(self, request, context):
        self._rt(request.bridge, context)
        return pb.GetPipeResponse(p4info_text=self.p4info_text.get(request.bridge or "br0", ""))

    def start(self, address: str = "127.0.0.1:0") -> "P4rtServer":
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        self._server.add_generic_rpc_handlers((service_handler(pb, "P4rt", self),))
        self.port = self._server.add_insecure_port(address)
        if not self.port:
            raise OSError(f"cannot bind the pipeline server on {address}")
        self._server.start()
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=0.2)
            self._server = None


def entry_text(info: P4Info, e) -> str:
    t = info.table(e.table)
    parts = []
    for (f, v, m), mf in zip(e.key, t.match_fields):
        full = (1 << mf.bitwidth) - 1
        parts.append(f"{f}={v:#x}" + (f"/{m:#x}" if mf.match_type != "EXACT" else ""))
    if e.priority:
        parts.append(f"priority={e.priority}")
    args = ",".join(f"{k}={v}" for k, v in e.params.items())
    parts.append(f"action={e.action}({args})")
    return ",".join(parts)


# ------------------------------------------------------------------------------------------ clients
@dataclass
class RuleResult:
    ok: bool
    stdout: str = ""
    stderr: str = ""


class P4rtClient:
    def run(self, verb: str, bridge: str, table: str, entry: str) -> RuleResult: ...


class GrpcP4rtClient(P4rtClient):
    def __init__(self, target: str):
        self.channel = grpc.insecure_channel(target)
        self.stub = Stub(self.channel, pb, "P4rt")

    def run(self, verb, bridge, table, entry):
        typ = {"add-entry": pb.INSERT, "del-entry": pb.DELETE, "mod-entry": pb.MODIFY}[verb]
        try:
            self.stub.Write(pb.WriteRequest(bridge=bridge, updates=[pb.Update(type=typ, table=table, entry=entry)]),
                            timeout=10)
            return RuleResult(True)
        except grpc.RpcError as e:
            return RuleResult(False, e.details() or "", e.details() or "")

    def close(self) -> None:
        self.channel.close()


class InProcessP4rtClient(P4rtClient):
    def __init__(self, runtimes: dict[str, P4Runtime]):
        self.runtimes = runtimes

    def run(self, verb, bridge, table, entry):
        rt = self.runtimes[bridge]
        try:
            if verb == "add-entry":
                rt.add_entry(table, entry)
            elif verb == "del-entry":
                rt.del_entry(table, entry)
            else:
                raise P4Error("INVALID_ARGUMENT", f"unknown verb {verb}")
            return RuleResult(True)
        except P4Error as e:
            return RuleResult(False, str(e), str(e))


class CliP4rtClient(P4rtClient):
    """`p4rt-ctl -g <ip:port> <verb> <bridge> <table> <entry>` through a Runner."""

    _mu = threading.Lock()

    def __init__(self, runner, ip_port: str, argv0: list[str] | None = None):
        self.runner = runner
        self.ip_port = ip_port
        self.argv0 = argv0 or ["python3", "-m", "dpu_operator_amd.cmd.p4rt_ctl"]

    def run(self, verb, bridge, table, entry):
        from ..utils.cmdrunner import CommandError

        with self._mu:
            try:
                out = self.runner.run([*self.argv0, "-g", self.ip_port, verb, bridge, table, entry])
                return RuleResult(True, out)
            except CommandError as e:
                return RuleResult(False, e.out, e.out)


@dataclass
class Rule:
    verb: str      # add-entry / del-entry
    bridge: str
    table: str
    entry: str


def program_rules(client: P4rtClient, rules: list[Rule]) -> list[Rule]:
    """ProgramFXPP4Rules (p4rtclient.go:74-101) -> rules that still failed."""
    failed = []
    for r in rules:
        res = client.run(r.verb, r.bridge, r.table, r.entry)
        if res.ok:
            continue
        if "ALREADY_EXISTS" in res.stdout:
            key = r.entry[: r.entry.index(",action")] if ",action" in r.entry else r.entry
            client.run("del-entry", r.bridge, r.table, key)
            res = client.run(r.verb, r.bridge, r.table, r.entry)
        elif "INVALID_ARGUMENT" in res.stderr:
            res = client.run(r.verb, r.bridge, r.table, r.entry)
        if not res.ok:
            log.warning("p4 rule failed: %s %s %s: %s", r.verb, r.table, r.entry, res.stderr.strip())
            failed.append(r)
    return failed


__all__ = ["P4rtServer", "GrpcP4rtClient", "CliP4rtClient", "InProcessP4rtClient", "Rule", "program_rules",
           "entry_text", "MI355X_P4INFO"]
