"""gRPC plumbing for descriptor-built services: generic server handlers and client stubs.

`serve(service_ns, service, impl)` builds a ``grpc.GenericRpcHandler`` from an object exposing one
Python method per RPC (snake_case or the proto name); `Stub(channel, ns, service)` exposes the
RPCs as callables.  Unary and server-streaming RPCs are supported (the device plugin's
ListAndWatch is server-streaming).
"""
from __future__ import annotations

import re

import grpc


def _snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def service_handler(ns, service: str, impl) -> grpc.GenericRpcHandler:
    handlers = {}
    for meth, (req_t, resp_t, stream) in ns.methods(service).items():
        fn = getattr(impl, meth, None) or getattr(impl, _snake(meth), None)
        if fn is None:
            def fn(request, context, _m=meth):  # noqa: ANN001
                context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{_m} not implemented")
        if stream:
            handlers[meth] = grpc.unary_stream_rpc_method_handler(
                fn, request_deserializer=req_t.FromString, response_serializer=resp_t.SerializeToString)
        else:
            handlers[meth] = grpc.unary_unary_rpc_method_handler(
                fn, request_deserializer=req_t.FromString, response_serializer=resp_t.SerializeToString)
    return grpc.method_handlers_generic_handler(f"{ns.package}.{service}", handlers)


class Stub:
    def __init__(self, channel: grpc.Channel, ns, service: str):
        for meth, (req_t, resp_t, stream) in ns.methods(service).items():
            path = ns.method_path(service, meth)
            if stream:
                call = channel.unary_stream(path, request_serializer=req_t.SerializeToString,
                                            response_deserializer=resp_t.FromString)
            else:
                call = channel.unary_unary(path, request_serializer=req_t.SerializeToString,
                                           response_deserializer=resp_t.FromString)
            setattr(self, meth, call)


def retry_service_config(max_attempts: int = 40, initial: str = "1s", max_backoff: str = "16s") -> str:
    """The reference's client retry policy: UNAVAILABLE retried with exponential backoff
    (internal/daemon/hostsidemanager.go:154-166; gRPC caps maxAttempts at 5 unless raised)."""
    import json

    return json.dumps({
        "methodConfig": [{
            "name": [{}],
            "waitForReady": True,
            "retryPolicy": {"maxAttempts": max_attempts, "initialBackoff": initial, "maxBackoff": max_backoff,
                            "backoffMultiplier": 2.0, "retryableStatusCodes": ["UNAVAILABLE"]},
        }]
    })


def unix_target(path: str) -> str:
    return f"unix://{path}"
