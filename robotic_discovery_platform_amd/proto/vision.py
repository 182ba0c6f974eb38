"""``evofab.vision`` wire contract, built at runtime (no protoc in the image).

Schema = ``/root/reference/protos/vision.proto:1-41`` (package ``evofab.vision``; ``Point3D``, ``Image``,
``AnalysisRequest``, ``AnalysisResponse``; service ``VisionAnalysisService`` with the stream->stream
RPC ``AnalyzeActuatorPerformance``). The descriptor is assembled field by field with
``descriptor_pb2`` so the encoding is byte-identical to the reference's generated ``vision_pb2``
(golden vectors: SURVEY.md App. A, tests/test_proto_wire.py). The gRPC glue
(``VisionAnalysisServiceStub`` / ``add_VisionAnalysisServiceServicer_to_server``) mirrors the surface
of ``pkg/protos/vision_pb2_grpc.py:28-68`` via grpc's generic handlers.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "evofab.vision"
SERVICE = "VisionAnalysisService"
METHOD = "AnalyzeActuatorPerformance"
FULL_SERVICE = f"{PACKAGE}.{SERVICE}"
METHOD_PATH = f"/{FULL_SERVICE}/{METHOD}"

_F = descriptor_pb2.FieldDescriptorProto


def _file_proto() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="vision.proto", package=PACKAGE, syntax="proto3")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label, json_name=_camel(fname))
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"

    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    msg("Point3D", [("x", 1, _F.TYPE_DOUBLE, opt, None), ("y", 2, _F.TYPE_DOUBLE, opt, None),
                    ("z", 3, _F.TYPE_DOUBLE, opt, None)])
    msg("Image", [("data", 1, _F.TYPE_BYTES, opt, None), ("width", 2, _F.TYPE_INT32, opt, None),
                  ("height", 3, _F.TYPE_INT32, opt, None)])
    msg("AnalysisRequest", [("color_image", 1, _F.TYPE_MESSAGE, opt, "Image"),
                            ("depth_image", 2, _F.TYPE_MESSAGE, opt, "Image")])
    msg("AnalysisResponse", [("mean_curvature", 1, _F.TYPE_DOUBLE, opt, None),
                             ("max_curvature", 2, _F.TYPE_DOUBLE, opt, None),
                             ("spline_points", 3, _F.TYPE_MESSAGE, rep, "Point3D"),
                             ("status", 4, _F.TYPE_STRING, opt, None),
                             ("mask", 5, _F.TYPE_BYTES, opt, None),
                             ("mask_coverage", 6, _F.TYPE_FLOAT, opt, None),
                             ("proc_time_ms", 7, _F.TYPE_FLOAT, opt, None)])
    svc = fd.service.add(name=SERVICE)
    svc.method.add(name=METHOD, input_type=f".{PACKAGE}.AnalysisRequest", output_type=f".{PACKAGE}.AnalysisResponse",
                   client_streaming=True, server_streaming=True)
    return fd


def _camel(s: str) -> str:
    head, *rest = s.split("_")
    return head + "".join(w.capitalize() for w in rest)


_POOL = descriptor_pool.DescriptorPool()
FILE_DESCRIPTOR = _POOL.Add(_file_proto())
DESCRIPTOR = _POOL.FindFileByName("vision.proto")

Point3D = message_factory.GetMessageClass(DESCRIPTOR.message_types_by_name["Point3D"])
Image = message_factory.GetMessageClass(DESCRIPTOR.message_types_by_name["Image"])
AnalysisRequest = message_factory.GetMessageClass(DESCRIPTOR.message_types_by_name["AnalysisRequest"])
AnalysisResponse = message_factory.GetMessageClass(DESCRIPTOR.message_types_by_name["AnalysisResponse"])


# ----------------------------------------------------------------------------- gRPC glue
class VisionAnalysisServiceStub:
    """Client stub: ``stub.AnalyzeActuatorPerformance(request_iterator) -> response iterator``."""

    def __init__(self, channel):
        self.AnalyzeActuatorPerformance = channel.stream_stream(
            METHOD_PATH, request_serializer=AnalysisRequest.SerializeToString,
            response_deserializer=AnalysisResponse.FromString)


class VisionAnalysisServiceServicer:
    def AnalyzeActuatorPerformance(self, request_iterator, context):  # pragma: no cover - interface
        import grpc
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")


def _serialize_response(m) -> bytes:
    """A response message, or its wire bytes already encoded (the server's native fast path)."""
    return m if isinstance(m, (bytes, bytearray)) else m.SerializeToString()


def add_VisionAnalysisServiceServicer_to_server(servicer, server) -> None:
    """A servicer with ``raw_requests`` true receives each request as its serialized bytes (the native
    serving path reads the two image payloads in place, csrc/serve_runtime.cpp parse_request, and parses
    with AnalysisRequest.FromString only the frames it hands back); otherwise AnalysisRequest messages."""
    import grpc
    raw = bool(getattr(servicer, "raw_requests", False))
    handlers = {
        METHOD: grpc.stream_stream_rpc_method_handler(
            servicer.AnalyzeActuatorPerformance, request_deserializer=None if raw else AnalysisRequest.FromString,
            response_serializer=_serialize_response),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(FULL_SERVICE, handlers),))
