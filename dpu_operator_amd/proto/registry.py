"""Protocol Buffers for the three gRPC surfaces, built from hand-written descriptors.

No protoc in this environment: message classes are generated at import time from
``FileDescriptorProto``s (same package names, message names, field numbers and types as the
reference's .proto files), so the wire bytes and the full RPC method paths are identical:

* ``Vendor`` (dpu-api/api.proto:1-54): LifeCycleService.Init, NetworkFunctionService.
  {Create,Delete}NetworkFunction, DeviceService.{GetDevices,SetNumVfs}
* ``opi_api.network.evpn_gw.v1alpha1`` BridgePortService / LogicalBridgeService subset
  (vendor/github.com/opiproject/opi-api/.../l2_xpu_infra_mgr.pb.go field tags)
* ``v1beta1`` kubelet device plugin (vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto)
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, empty_pb2, field_mask_pb2, message_factory

F = descriptor_pb2.FieldDescriptorProto
_SCALARS = {
    "double": F.TYPE_DOUBLE, "float": F.TYPE_FLOAT, "int64": F.TYPE_INT64, "uint64": F.TYPE_UINT64,
    "int32": F.TYPE_INT32, "uint32": F.TYPE_UINT32, "bool": F.TYPE_BOOL, "string": F.TYPE_STRING,
    "bytes": F.TYPE_BYTES,
}

POOL = descriptor_pool.DescriptorPool()
POOL.AddSerializedFile(empty_pb2.DESCRIPTOR.serialized_pb)
POOL.AddSerializedFile(field_mask_pb2.DESCRIPTOR.serialized_pb)


def _field(msg: descriptor_pb2.DescriptorProto, pkg: str, name: str, number: int, typ: str,
           repeated: bool = False, optional: bool = False, enum: bool = False) -> None:
    f = msg.field.add()
    f.name = name
    f.number = number
    f.label = F.LABEL_REPEATED if repeated else F.LABEL_OPTIONAL
    if typ in _SCALARS:
        f.type = _SCALARS[typ]
    else:
        f.type = F.TYPE_ENUM if enum else F.TYPE_MESSAGE
        f.type_name = typ if typ.startswith(".") else f".{pkg}.{typ}"
    f.json_name = "".join(p.capitalize() if i else p for i, p in enumerate(name.split("_")))
    if optional:  # proto3 `optional` -> synthetic oneof
        f.proto3_optional = True
        o = msg.oneof_decl.add()
        o.name = f"_{name}"
        f.oneof_index = len(msg.oneof_decl) - 1


def _map(msg: descriptor_pb2.DescriptorProto, pkg: str, name: str, number: int, ktype: str, vtype: str) -> None:
    entry = msg.nested_type.add()
    entry.name = "".join(p.capitalize() for p in name.split("_")) + "Entry"
    entry.options.map_entry = True
    _field(entry, pkg, "key", 1, ktype)
    _field(entry, pkg, "value", 2, vtype)
    f = msg.field.add()
    f.name, f.number, f.label, f.type = name, number, F.LABEL_REPEATED, F.TYPE_MESSAGE
    f.type_name = f".{pkg}.{msg.name}.{entry.name}"
    f.json_name = "".join(p.capitalize() if i else p for i, p in enumerate(name.split("_")))


def _build(fname: str, pkg: str, messages: dict, services: dict, enums: dict | None = None,
           deps: tuple = ()) -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name=fname, package=pkg, syntax="proto3")
    fd.dependency.extend(deps)
    for ename, values in (enums or {}).items():
        e = fd.enum_type.add(name=ename)
        for vname, num in values:
            e.value.add(name=vname, number=num)
    for mname, fields in messages.items():
        m = fd.message_type.add(name=mname)
        for spec in fields:
            kind = spec[0]
            if kind == "map":
                _, name, num, kt, vt = spec
                _map(m, pkg, name, num, kt, vt)
            else:
                name, num, typ, *flags = spec
                _field(m, pkg, name, num, typ, repeated="repeated" in flags, optional="optional" in flags,
                       enum="enum" in flags)
    for sname, methods in services.items():
        s = fd.service.add(name=sname)
        for meth, (inp, out, *flags) in methods.items():
            md = s.method.add(name=meth)
            md.input_type = inp if inp.startswith(".") else f".{pkg}.{inp}"
            md.output_type = out if out.startswith(".") else f".{pkg}.{out}"
            md.server_streaming = "stream" in flags
    return fd


# ---------------------------------------------------------------------------- dpu-api (Vendor)
VENDOR_FILE = _build(
    "dpu-api/api.proto", "Vendor",
    messages={
        "InitRequest": [("dpu_mode", 1, "bool"), ("dpu_identifier", 2, "string")],
        "IpPort": [("ip", 1, "string"), ("port", 2, "int32")],
        "NFRequest": [("input", 1, "string"), ("output", 2, "string")],
        "Empty": [],
        "VfCount": [("vf_cnt", 1, "int32")],
        "TopologyInfo": [("node", 1, "string")],
        "Device": [("ID", 1, "string"), ("health", 2, "string"), ("topology", 3, "TopologyInfo")],
        "DeviceListResponse": [("map", "devices", 1, "string", ".Vendor.Device")],
    },
    services={
        "LifeCycleService": {"Init": ("InitRequest", "IpPort")},
        "NetworkFunctionService": {"CreateNetworkFunction": ("NFRequest", "Empty"),
                                   "DeleteNetworkFunction": ("NFRequest", "Empty")},
        "DeviceService": {"GetDevices": ("Empty", "DeviceListResponse"), "SetNumVfs": ("VfCount", "VfCount")},
    },
)

# ---------------------------------------------------------------------------- OPI evpn-gw subset
OPI_PKG = "opi_api.network.evpn_gw.v1alpha1"
OPI_FILE = _build(
    "opi/l2_xpu_infra_mgr.proto", OPI_PKG,
    enums={
        "BridgePortType": [("BRIDGE_PORT_TYPE_UNSPECIFIED", 0), ("BRIDGE_PORT_TYPE_ACCESS", 1),
                           ("BRIDGE_PORT_TYPE_TRUNK", 2)],
        "BPOperStatus": [("BP_OPER_STATUS_UNSPECIFIED", 0), ("BP_OPER_STATUS_UP", 1), ("BP_OPER_STATUS_DOWN", 2),
                         ("BP_OPER_STATUS_TO_BE_DELETED", 3)],
        "LBOperStatus": [("LB_OPER_STATUS_UNSPECIFIED", 0), ("LB_OPER_STATUS_UP", 1), ("LB_OPER_STATUS_DOWN", 2),
                         ("LB_OPER_STATUS_TO_BE_DELETED", 3)],
        "CompStatus": [("COMP_STATUS_UNSPECIFIED", 0), ("COMP_STATUS_PENDING", 1), ("COMP_STATUS_SUCCESS", 2),
                       ("COMP_STATUS_ERROR", 3)],
    },
    messages={
        "Component": [("name", 1, "string"), ("status", 2, "CompStatus", "enum"), ("details", 3, "string")],
        "BridgePortSpec": [("mac_address", 1, "bytes"), ("ptype", 2, "BridgePortType", "enum"),
                           ("logical_bridges", 3, "string", "repeated")],
        "BridgePortStatus": [("oper_status", 1, "BPOperStatus", "enum"), ("components", 2, "Component", "repeated")],
        "BridgePort": [("name", 1, "string"), ("spec", 2, "BridgePortSpec"), ("status", 3, "BridgePortStatus")],
        "CreateBridgePortRequest": [("bridge_port_id", 1, "string"), ("bridge_port", 2, "BridgePort")],
        "ListBridgePortsRequest": [("page_size", 1, "int32"), ("page_token", 2, "string")],
        "ListBridgePortsResponse": [("bridge_ports", 1, "BridgePort", "repeated"), ("next_page_token", 2, "string")],
        "GetBridgePortRequest": [("name", 1, "string")],
        "DeleteBridgePortRequest": [("name", 1, "string"), ("allow_missing", 2, "bool")],
        "UpdateBridgePortRequest": [("bridge_port", 1, "BridgePort"), ("update_mask", 2, ".google.protobuf.FieldMask"),
                                    ("allow_missing", 3, "bool")],
        "LogicalBridgeSpec": [("vlan_id", 1, "uint32"), ("vni", 2, "uint32", "optional")],
        "LogicalBridgeStatus": [("oper_status", 1, "LBOperStatus", "enum"), ("components", 2, "Component", "repeated")],
        "LogicalBridge": [("name", 1, "string"), ("spec", 2, "LogicalBridgeSpec"), ("status", 3, "LogicalBridgeStatus")],
        "CreateLogicalBridgeRequest": [("logical_bridge_id", 1, "string"), ("logical_bridge", 2, "LogicalBridge")],
        "GetLogicalBridgeRequest": [("name", 1, "string")],
        "DeleteLogicalBridgeRequest": [("name", 1, "string"), ("allow_missing", 2, "bool")],
        "ListLogicalBridgesRequest": [("page_size", 1, "int32"), ("page_token", 2, "string")],
        "ListLogicalBridgesResponse": [("logical_bridges", 1, "LogicalBridge", "repeated"),
                                       ("next_page_token", 2, "string")],
    },
    services={
        "BridgePortService": {
            "CreateBridgePort": ("CreateBridgePortRequest", "BridgePort"),
            "ListBridgePorts": ("ListBridgePortsRequest", "ListBridgePortsResponse"),
            "GetBridgePort": ("GetBridgePortRequest", "BridgePort"),
            "DeleteBridgePort": ("DeleteBridgePortRequest", ".google.protobuf.Empty"),
            "UpdateBridgePort": ("UpdateBridgePortRequest", "BridgePort"),
        },
        "LogicalBridgeService": {
            "CreateLogicalBridge": ("CreateLogicalBridgeRequest", "LogicalBridge"),
            "ListLogicalBridges": ("ListLogicalBridgesRequest", "ListLogicalBridgesResponse"),
            "GetLogicalBridge": ("GetLogicalBridgeRequest", "LogicalBridge"),
            "DeleteLogicalBridge": ("DeleteLogicalBridgeRequest", ".google.protobuf.Empty"),
        },
    },
    deps=("google/protobuf/empty.proto", "google/protobuf/field_mask.proto"),
)

# ---------------------------------------------------------------------------- kubelet v1beta1
DP_FILE = _build(
    "deviceplugin/v1beta1/api.proto", "v1beta1",
    messages={
        "DevicePluginOptions": [("pre_start_required", 1, "bool"), ("get_preferred_allocation_available", 2, "bool")],
        "RegisterRequest": [("version", 1, "string"), ("endpoint", 2, "string"), ("resource_name", 3, "string"),
                            ("options", 4, "DevicePluginOptions")],
        "Empty": [],
        "ListAndWatchResponse": [("devices", 1, "Device", "repeated")],
        "NUMANode": [("ID", 1, "int64")],
        "TopologyInfo": [("nodes", 1, "NUMANode", "repeated")],
        "Device": [("ID", 1, "string"), ("health", 2, "string"), ("topology", 3, "TopologyInfo")],
        "PreStartContainerRequest": [("devices_ids", 1, "string", "repeated")],
        "PreStartContainerResponse": [],
        "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, "string", "repeated"),
                                                ("must_include_deviceIDs", 2, "string", "repeated"),
                                                ("allocation_size", 3, "int32")],
        "PreferredAllocationRequest": [("container_requests", 1, "ContainerPreferredAllocationRequest", "repeated")],
        "ContainerPreferredAllocationResponse": [("deviceIDs", 1, "string", "repeated")],
        "PreferredAllocationResponse": [("container_responses", 1, "ContainerPreferredAllocationResponse", "repeated")],
        "ContainerAllocateRequest": [("devices_ids", 1, "string", "repeated")],
        "AllocateRequest": [("container_requests", 1, "ContainerAllocateRequest", "repeated")],
        "CDIDevice": [("name", 1, "string")],
        "Mount": [("container_path", 1, "string"), ("host_path", 2, "string"), ("read_only", 3, "bool")],
        "DeviceSpec": [("container_path", 1, "string"), ("host_path", 2, "string"), ("permissions", 3, "string")],
        "ContainerAllocateResponse": [("map", "envs", 1, "string", "string"), ("mounts", 2, "Mount", "repeated"),
                                      ("devices", 3, "DeviceSpec", "repeated"),
                                      ("map", "annotations", 4, "string", "string"),
                                      ("cdi_devices", 5, "CDIDevice", "repeated")],
        "AllocateResponse": [("container_responses", 1, "ContainerAllocateResponse", "repeated")],
    },
    services={
        "Registration": {"Register": ("RegisterRequest", "Empty")},
        "DevicePlugin": {
            "GetDevicePluginOptions": ("Empty", "DevicePluginOptions"),
            "ListAndWatch": ("Empty", "ListAndWatchResponse", "stream"),
            "GetPreferredAllocation": ("PreferredAllocationRequest", "PreferredAllocationResponse"),
            "Allocate": ("AllocateRequest", "AllocateResponse"),
            "PreStartContainer": ("PreStartContainerRequest", "PreStartContainerResponse"),
        },
    },
)

# ---------------------------------------------------------------- MI355X P4 runtime (p4rt-ctl server)
# The reference's p4rt-ctl speaks P4Runtime to infrap4d; this framework's pipeline server takes
# the same rule strings in a small service (bridge + table + entry text), so p4rt-ctl semantics
# (ALREADY_EXISTS / NOT_FOUND / INVALID_ARGUMENT in the error text) carry over unchanged.
P4RT_FILE = _build(
    "mi355x/p4rt.proto", "mi355x.p4rt.v1",
    enums={"UpdateType": [("UNSPECIFIED", 0), ("INSERT", 1), ("MODIFY", 2), ("DELETE", 3)]},
    messages={
        "Update": [("type", 1, "UpdateType", "enum"), ("table", 2, "string"), ("entry", 3, "string")],
        "WriteRequest": [("bridge", 1, "string"), ("updates", 2, "Update", "repeated")],
        "WriteResponse": [("applied", 1, "int32")],
        "ReadRequest": [("bridge", 1, "string"), ("table", 2, "string")],
        "TableEntry": [("table", 1, "string"), ("entry", 2, "string")],
        "ReadResponse": [("entries", 1, "TableEntry", "repeated")],
        "SetPipeRequest": [("bridge", 1, "string"), ("p4info_text", 2, "string")],
        "SetPipeResponse": [("tables", 1, "int32"), ("actions", 2, "int32")],
        "GetPipeRequest": [("bridge", 1, "string")],
        "GetPipeResponse": [("p4info_text", 1, "string")],
    },
    services={"P4rt": {"Write": ("WriteRequest", "WriteResponse"), "Read": ("ReadRequest", "ReadResponse"),
                       "SetPipe": ("SetPipeRequest", "SetPipeResponse"),
                       "GetPipe": ("GetPipeRequest", "GetPipeResponse")}},
)

for _fd in (VENDOR_FILE, OPI_FILE, DP_FILE, P4RT_FILE):
    POOL.Add(_fd)


class _Namespace:
    def __init__(self, pkg: str, fd: descriptor_pb2.FileDescriptorProto):
        self.package = pkg
        self.file = fd
        for m in fd.message_type:
            setattr(self, m.name, message_factory.GetMessageClass(POOL.FindMessageTypeByName(f"{pkg}.{m.name}")))
        for e in fd.enum_type:
            ed = POOL.FindEnumTypeByName(f"{pkg}.{e.name}")
            for v in ed.values:
                setattr(self, v.name, v.number)

    def method_path(self, service: str, method: str) -> str:
        return f"/{self.package}.{service}/{method}"

    def methods(self, service: str) -> dict[str, tuple[type, type, bool]]:
        sd = POOL.FindServiceByName(f"{self.package}.{service}")
        out = {}
        for md in sd.methods:
            out[md.name] = (message_factory.GetMessageClass(md.input_type),
                            message_factory.GetMessageClass(md.output_type), md.server_streaming)
        return out


vendor = _Namespace("Vendor", VENDOR_FILE)
opi = _Namespace(OPI_PKG, OPI_FILE)
deviceplugin = _Namespace("v1beta1", DP_FILE)
p4rt = _Namespace("mi355x.p4rt.v1", P4RT_FILE)
GoogleEmpty = message_factory.GetMessageClass(POOL.FindMessageTypeByName("google.protobuf.Empty"))

HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"
DEVICE_PLUGIN_VERSION = "v1beta1"
