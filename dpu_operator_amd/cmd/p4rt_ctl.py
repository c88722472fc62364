"""`p4rt-ctl` — control the MI355X pipeline server's P4 bridges.

Reference: cmd/intelvsp/p4rt-ctl (usage :53-80).  Commands kept: show, set-pipe,
get-pipe, add-entry, mod-entry, del-entry, dump-entries; `-g host:port` selects the server
(default 127.0.0.1:9559).  Entry syntax is the reference's: `field=value[/mask],...,priority=N,
action=ctrl.action(arg,...)`; keys for del-entry omit the action.  Failures print the P4Runtime
code (ALREADY_EXISTS, NOT_FOUND, INVALID_ARGUMENT, ...) on stdout and stderr and exit 1.
Packet-IO and meter commands of the IPU tool have no MI355X pipeline counterpart.
"""
from __future__ import annotations

import argparse
import sys

import grpc

from ..proto import p4rt as pb
from ..proto.grpcutil import Stub

DEFAULT_TARGET = "127.0.0.1:9559"


def _fail(e: grpc.RpcError) -> int:
    msg = e.details() or str(e.code())
    print(msg)
    print(msg, file=sys.stderr)
    return 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="p4rt-ctl", description="control P4 bridges of the MI355X pipeline server")
    ap.add_argument("-g", "--grpc-addr", default=DEFAULT_TARGET)
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("show")
    s.add_argument("switch")
    s = sub.add_parser("set-pipe")
    s.add_argument("switch")
    s.add_argument("program", help="pipeline binary (ignored: the GPU pipeline is built in)")
    s.add_argument("p4info")
    s = sub.add_parser("get-pipe")
    s.add_argument("switch")
    for verb in ("add-entry", "mod-entry"):
        s = sub.add_parser(verb)
        s.add_argument("switch")
        s.add_argument("table")
        s.add_argument("flow")
    s = sub.add_parser("del-entry")
    s.add_argument("switch")
    s.add_argument("table")
    s.add_argument("key")
    s = sub.add_parser("dump-entries")
    s.add_argument("switch")
    s.add_argument("table", nargs="?", default="")
    a = ap.parse_args(argv)
    ch = grpc.insecure_channel(a.grpc_addr)
    stub = Stub(ch, pb, "P4rt")
    try:
        if a.cmd in ("add-entry", "mod-entry", "del-entry"):
            typ = {"add-entry": pb.INSERT, "mod-entry": pb.MODIFY, "del-entry": pb.DELETE}[a.cmd]
            entry = a.key if a.cmd == "del-entry" else a.flow
            stub.Write(pb.WriteRequest(bridge=a.switch, updates=[pb.Update(type=typ, table=a.table, entry=entry)]),
                       timeout=10)
        elif a.cmd == "dump-entries":
            for e in stub.Read(pb.ReadRequest(bridge=a.switch, table=a.table), timeout=10).entries:
                print(f"{e.table} {e.entry}")
        elif a.cmd == "set-pipe":
            with open(a.p4info) as f:
                r = stub.SetPipe(pb.SetPipeRequest(bridge=a.switch, p4info_text=f.read()), timeout=30)
            print(f"pipeline set: {r.tables} tables, {r.actions} actions")
        elif a.cmd == "get-pipe":
            print(stub.GetPipe(pb.GetPipeRequest(bridge=a.switch), timeout=10).p4info_text, end="")
        elif a.cmd == "show":
            r = stub.Read(pb.ReadRequest(bridge=a.switch), timeout=10)
            counts: dict[str, int] = {}
            for e in r.entries:
                counts[e.table] = counts.get(e.table, 0) + 1
            print(f"P4Runtime switch {a.switch} ({len(r.entries)} entries)")
            for t, n in sorted(counts.items()):
                print(f"  {t}: {n}")
    except grpc.RpcError as e:
        return _fail(e)
    finally:
        ch.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
