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
