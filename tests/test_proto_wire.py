"""Wire compatibility of the runtime-built evofab.vision descriptor (golden vectors: SURVEY.md App. A,
generated from the reference's checked-in descriptor /root/reference/pkg/protos/vision_pb2.py:27)."""
from robotic_discovery_platform_amd.proto import vision as pb

GOLD = [
    (lambda: pb.AnalysisRequest(color_image=pb.Image(data=b"\xff\xd8", width=640, height=480),
                                depth_image=pb.Image(data=b"\x89P", width=640, height=480)),
     "0a0a0a02ffd810800518e003120a0a02895010800518e003"),
    (lambda: pb.AnalysisResponse(mean_curvature=1.5, mask=b"ab", proc_time_ms=3.0,
                                 spline_points=[pb.Point3D(x=1, y=2, z=3)]),
     "09000000000000f83f1a1b09000000000000f03f1100000000000000401900000000000008402a0261623d00004040"),
    (lambda: pb.AnalysisResponse(mean_curvature=0.25, max_curvature=2.0, status="ok", mask=b"\x00",
                                 mask_coverage=12.5, proc_time_ms=1.5,
                                 spline_points=[pb.Point3D(x=0.1, y=-0.2, z=0.6)]),
     "09000000000000d03f1100000000000000401a1b099a9999999999b93f119a9999999999c9bf19333333333333e33f"
     "22026f6b2a010035000048413d0000c03f"),
    (lambda: pb.AnalysisResponse(), ""),
]


def test_golden_serialize():
    for make, hexs in GOLD:
        assert make().SerializeToString().hex() == hexs


def test_golden_parse_roundtrip():
    for make, hexs in GOLD:
        m = make()
        back = type(m).FromString(bytes.fromhex(hexs))
        assert back == m


def test_service_shape():
    svc = pb.DESCRIPTOR.services_by_name["VisionAnalysisService"]
    meth = svc.methods_by_name["AnalyzeActuatorPerformance"]
    assert meth.client_streaming and meth.server_streaming
    assert pb.METHOD_PATH == "/evofab.vision.VisionAnalysisService/AnalyzeActuatorPerformance"
    assert pb.DESCRIPTOR.package == "evofab.vision"


def test_native_request_parser_matches_protobuf():
    """csrc/serve_runtime.cpp parse_request (the server's raw-bytes fast path) extracts the same image
    payloads protobuf does -- field order, unknown fields, repeated fields (last wins) -- and declines
    what it does not take (missing image, truncated bytes) so the server falls back to protobuf."""
    import random
    from robotic_discovery_platform_amd.ops import native
    from robotic_discovery_platform_amd.proto import vision as pb
    C = native(build_if_missing=False)
    rng = random.Random(3)
    for trial in range(50):
        c = bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 3000)))
        d = bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 5000)))
        req = pb.AnalysisRequest(color_image=pb.Image(data=c, width=rng.randint(0, 9999), height=640),
                                 depth_image=pb.Image(data=d, width=640, height=rng.randint(0, 9999)))
        raw = req.SerializeToString()
        if trial % 3 == 1:  # depth first on the wire
            raw = (pb.AnalysisRequest(depth_image=req.depth_image).SerializeToString() +
                   pb.AnalysisRequest(color_image=req.color_image).SerializeToString())
        if trial % 3 == 2:  # an unknown field (number 9, varint) and a stale colour payload before the real one
            raw = b"\x48\x07" + pb.AnalysisRequest(color_image=pb.Image(data=b"old")).SerializeToString() + raw
        got = C.parse_request(raw)
        msg = pb.AnalysisRequest.FromString(raw)
        assert got == (msg.color_image.data, msg.depth_image.data)
    only_color = pb.AnalysisRequest(color_image=pb.Image(data=b"x")).SerializeToString()
    assert C.parse_request(only_color) is None
    full = pb.AnalysisRequest(color_image=pb.Image(data=b"abc"), depth_image=pb.Image(data=b"def")).SerializeToString()
    assert C.parse_request(full[:-2]) is None
