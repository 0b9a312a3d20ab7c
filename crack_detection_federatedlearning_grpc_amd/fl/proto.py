"""``transport.proto`` built at import time from a hand-written FileDescriptorProto.

The reference imports generated ``transport_pb2`` / ``transport_pb2_grpc`` (fl_server.py:8-9, fl_client.py:8-9)
whose ``.proto`` is missing from the snapshot; ``protoc``/``grpcio-tools`` are not available here, so the schema
reconstructed in SURVEY.md §2.4 is declared directly as descriptors. The human-readable schema is kept in
``proto/transport.proto`` and a test checks the two agree.

Field and enum names follow the reference's usage:
  ReadyReq{type,cname,state,config}          fl_client.py:27
  UpdateReq{type,buffer_chunk,title,file_len,cname,state,current_round}   fl_client.py:15,43,56,63
  UpdateRep{type,buffer_chunk,title,config}  fl_server.py:161,167,173,186-194
  VersionReq{type,config} / VersionRep{state,buffer_chunk,config}  fl_client.py:72, fl_server.py:201-207
  State{ON,TRAINING,TRAIN_DONE,WAIT,NOT_WAIT,FIN}   (FIN is needed because fl_server.py:145 puts it in .state)
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf.internal.enum_type_wrapper import EnumTypeWrapper

PACKAGE = "transport"
SERVICE = f"{PACKAGE}.TransportService"
METHOD = f"/{SERVICE}/transport"

_F = descriptor_pb2.FieldDescriptorProto
_STATES = ["ON", "TRAINING", "TRAIN_DONE", "WAIT", "NOT_WAIT", "FIN"]


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="transport.proto", package=PACKAGE, syntax="proto3")
    en = fd.enum_type.add(name="State")
    for i, s in enumerate(_STATES):
        en.value.add(name=s, number=i)

    def msg(name, fields, maps=()):
        m = fd.message_type.add(name=name)
        num = 1
        for fname, ftype, tname in fields:
            f = m.field.add(name=fname, number=num, label=_F.LABEL_OPTIONAL, type=ftype)
            if tname:
                f.type_name = tname
            num += 1
        for fname in maps:  # map<string, Scalar>
            entry = m.nested_type.add(name=fname[0].upper() + fname[1:] + "Entry")
            entry.options.map_entry = True
            entry.field.add(name="key", number=1, label=_F.LABEL_OPTIONAL, type=_F.TYPE_STRING)
            entry.field.add(name="value", number=2, label=_F.LABEL_OPTIONAL, type=_F.TYPE_MESSAGE,
                            type_name=f".{PACKAGE}.Scalar")
            m.field.add(name=fname, number=num, label=_F.LABEL_REPEATED, type=_F.TYPE_MESSAGE,
                        type_name=f".{PACKAGE}.{name}.{entry.name}")
            num += 1
        return m

    S, I32, I64, B, FL, E, M = (_F.TYPE_STRING, _F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_BYTES, _F.TYPE_FLOAT,
                                _F.TYPE_ENUM, _F.TYPE_MESSAGE)
    st = f".{PACKAGE}.State"
    msg("Scalar", [("scfloat", FL, None), ("scint32", I32, None), ("scstring", S, None)])
    msg("ReadyReq", [("type", S, None), ("cname", S, None), ("state", E, st)], maps=["config"])
    msg("ReadyRep", [], maps=["config"])
    msg("UpdateReq", [("type", S, None), ("buffer_chunk", B, None), ("title", S, None), ("file_len", I64, None),
                      ("cname", S, None), ("state", E, st), ("current_round", I32, None)])
    msg("UpdateRep", [("type", S, None), ("buffer_chunk", B, None), ("title", S, None)], maps=["config"])
    msg("VersionReq", [("type", S, None)], maps=["config"])
    msg("VersionRep", [("state", E, st), ("buffer_chunk", B, None)], maps=["config"])
    msg("transportRequest", [("ready_req", M, f".{PACKAGE}.ReadyReq"), ("update_req", M, f".{PACKAGE}.UpdateReq"),
                             ("version_req", M, f".{PACKAGE}.VersionReq")])
    msg("transportResponse", [("ready_rep", M, f".{PACKAGE}.ReadyRep"), ("update_rep", M, f".{PACKAGE}.UpdateRep"),
                              ("version_rep", M, f".{PACKAGE}.VersionRep")])
    svc = fd.service.add(name="TransportService")
    svc.method.add(name="transport", input_type=f".{PACKAGE}.transportRequest",
                   output_type=f".{PACKAGE}.transportResponse", client_streaming=True, server_streaming=True)
    return fd


FILE_PROTO = _build_file()
_pool = descriptor_pool.DescriptorPool()
DESCRIPTOR = _pool.Add(FILE_PROTO)


def _cls(name: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"{PACKAGE}.{name}"))


Scalar = _cls("Scalar")
ReadyReq = _cls("ReadyReq")
ReadyRep = _cls("ReadyRep")
UpdateReq = _cls("UpdateReq")
UpdateRep = _cls("UpdateRep")
VersionReq = _cls("VersionReq")
VersionRep = _cls("VersionRep")
transportRequest = _cls("transportRequest")
transportResponse = _cls("transportResponse")
State = EnumTypeWrapper(_pool.FindEnumTypeByName(f"{PACKAGE}.State"))
ON, TRAINING, TRAIN_DONE, WAIT, NOT_WAIT, FIN = (State.Value(s) for s in _STATES)


def to_proto_text() -> str:
    """Render the descriptor as .proto text (used to check proto/transport.proto stays in sync)."""
    lines = ['syntax = "proto3";', f"package {PACKAGE};", "", "enum State {"]
    for i, s in enumerate(_STATES):
        lines.append(f"  {s} = {i};")
    lines.append("}")
    tnames = {_F.TYPE_STRING: "string", _F.TYPE_INT32: "int32", _F.TYPE_INT64: "int64", _F.TYPE_BYTES: "bytes",
              _F.TYPE_FLOAT: "float"}
    for m in FILE_PROTO.message_type:
        lines.append("")
        lines.append(f"message {m.name} {{")
        maps = {n.name for n in m.nested_type}
        for f in m.field:
            if f.type_name.split(".")[-1] in maps:
                lines.append(f"  map<string, Scalar> {f.name} = {f.number};")
            elif f.type in (_F.TYPE_MESSAGE, _F.TYPE_ENUM):
                lines.append(f"  {f.type_name.split('.')[-1]} {f.name} = {f.number};")
            else:
                lines.append(f"  {tnames[f.type]} {f.name} = {f.number};")
        lines.append("}")
    lines.append("")
    lines.append("service TransportService {")
    lines.append("  rpc transport(stream transportRequest) returns (stream transportResponse);")
    lines.append("}")
    return "\n".join(lines) + "\n"
