"""Whole-model parity: the native (HIP kernel) U-Net vs the plain-torch fp32 reference U-Net."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.float().reshape(-1), b.float().reshape(-1)
    return (a @ b / (a.norm() * b.norm() + 1e-20)).item()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-20)).item()


@pytest.mark.parametrize("depth,size,bilinear,N", [(2, 64, True, 2), (4, 128, True, 2), (4, 96, True, 2),
                                                   (2, 64, False, 2), (4, 128, False, 2), (4, 72, False, 2),
                                                   # the bench's exact shape and kernel dispatch (256^2, N=64:
                                                   # ring / halo / igemm choice, split-K, 512-block wgrad grid)
                                                   (4, 256, True, 64), (4, 256, False, 16)])
def test_native_forward_backward_matches_reference(depth, size, bilinear, N):
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(0)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1, bilinear, 64, depth).to(dev)
    nat = UNetNative(3, 1, bilinear, 64, depth, device=dev, init_from=ref)
    x = torch.rand(N, 3, size, size, device=dev)
    t = (torch.rand(N, 1, size, size, device=dev) > 0.5).float()
    # reference sees the same bf16-rounded input
    xq = x.to(torch.bfloat16).float()
    ex = nat.executor(N, size, size, training=True)
    ex.set_input(x, t)
    ex.forward()
    ref.train()
    out = ref(xq)
    loss = F.binary_cross_entropy_with_logits(out, t)
    loss.backward()
    assert _rel(ex.logits_nchw(), out.detach()) < 0.08
    assert abs(ex.loss[0].item() - loss.item()) < 2e-2
    ex.backward()
    st = nat.store
    # yardstick: torch's own bf16 autocast run of the same step vs the fp32 reference
    ref16 = UNetRef(3, 1, bilinear, 64, depth).to(dev)
    ref16.load_state_dict(ref.state_dict())
    with torch.autocast("cuda", dtype=torch.bfloat16):
        o16 = ref16(xq)
    F.binary_cross_entropy_with_logits(o16.float(), t).backward()
    p16 = dict(ref16.named_parameters())
    report = []
    for name, p in ref.named_parameters():
        g = st.view(name, st.grad)
        c = _cos(g, p.grad)
        c16 = _cos(p16[name].grad, p.grad)
        report.append((name, round(c, 4), round(c16, 4)))
    print("\n".join(map(str, report)))
    # native bf16 must be about as close to fp32 as torch's own bf16 autocast is
    mean_c = sum(r[1] for r in report) / len(report)
    mean_c16 = sum(r[2] for r in report) / len(report)
    assert mean_c > mean_c16 - 0.02, (mean_c, mean_c16)
    for name, c, c16 in report:
        assert c > min(0.97, c16 - 0.1), (name, c, c16)
    # running stats updated identically (momentum 0.1, unbiased var)
    for name, b in ref.named_buffers():
        if name.endswith("running_mean") or name.endswith("running_var"):
            assert _rel(nat.buf(name), b) < 0.05, name
        if name.endswith("num_batches_tracked"):
            assert int(nat.buf(name).item()) == int(b.item())


def test_state_dict_roundtrip_reference_keys():
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    dev = torch.device("cuda")
    ref = UNetRef(3, 1)
    nat = UNetNative(3, 1, device=dev, init_from=ref)
    sd = nat.state_dict()
    assert list(sd.keys()) == list(ref.state_dict().keys())
    for k, v in ref.state_dict().items():
        assert sd[k].shape == v.shape and torch.equal(sd[k].cpu(), v), k
    ref2 = UNetRef(3, 1)
    nat.load_state_dict(ref2.state_dict())
    assert torch.equal(nat.state_dict()["up2.conv.double_conv.3.weight"].cpu(), ref2.state_dict()["up2.conv.double_conv.3.weight"])


def test_native_training_reduces_loss_and_graph_replay_matches():
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(0)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1)
    x = torch.rand(4, 3, 64, 64, device=dev)
    yy, xx = torch.meshgrid(torch.arange(64, device=dev), torch.arange(64, device=dev), indexing="ij")
    t = (((yy - 32) ** 2 + (xx - 32) ** 2) < 300).float().expand(4, 1, 64, 64).contiguous()
    x[:, 0] += t[:, 0] * 0.5
    losses = {}
    for graph in (False, True):
        nat = UNetNative(3, 1, device=dev, init_from=ref)
        tr = NativeTrainer(nat, 4, 64, 64, lr=1e-3, graph=graph)
        tr.set_batch(x, t)
        ls = []
        for _ in range(12):
            ls.append(tr.step()[0].item())
        losses[graph] = ls
        assert ls[-1] < ls[0] * 0.8, ls
    # eager and graph-replayed training are the same program
    assert max(abs(a - b) for a, b in zip(losses[False], losses[True])) < 1e-3


@pytest.mark.parametrize("bilinear,loss", [(True, "bce"), (False, "bce_dice")])
def test_plan_replay_bitwise_equals_eager(bilinear, loss, monkeypatch):
    """NativeTrainer plan mode (the step recorded once by the native runtime, then replayed from C++)
    is the eager program: losses and every parameter / Adam state bitwise equal to eager steps over 7
    steps with a new batch each step (eager warm-up, the recorded step, 4 replays), both decoders."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(3)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1, bilinear=bilinear)
    g = torch.Generator(device="cpu").manual_seed(5)
    batches = [(torch.rand(2, 3, 64, 96, generator=g), (torch.rand(2, 1, 64, 96, generator=g) > 0.5).float())
               for _ in range(7)]
    runs = {}
    for mode in ("eager", "plan"):
        plan = mode != "eager"
        nat = UNetNative(3, 1, bilinear=bilinear, device=dev, init_from=ref)
        tr = NativeTrainer(nat, 2, 64, 96, lr=1e-3, loss=loss, plan=plan)
        assert tr.use_plan == plan
        ls = []
        for x, y in batches:
            tr.set_batch(x.to(dev), y.to(dev))
            ls.append(tr.step().clone())
        torch.cuda.synchronize()
        if plan:
            assert tr.plan_id is not None
        st = nat.store
        runs[mode] = (torch.stack(ls), st.flat.clone(), st.exp_avg.clone(), st.exp_avg_sq.clone(),
                      nat.derived.clone(), [b.clone() for _, b in nat.named_buffers()])
    a = runs["eager"]
    for mode in ("plan",):
        b = runs[mode]
        for u, v in zip(a[:5], b[:5]):
            assert torch.equal(u, v), mode
        for u, v in zip(a[5], b[5]):
            assert torch.equal(u, v), mode


def test_plan_rerecords_after_load_state_dict():
    """load_state_dict re-lays out the derived weights: a recorded plan is dropped and re-recorded, so
    the next steps use the loaded weights (same losses as a fresh eager trainer from that state)."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(4)
    dev = torch.device("cuda")
    x = torch.rand(2, 3, 64, 64, device=dev)
    y = (torch.rand(2, 1, 64, 64, device=dev) > 0.5).float()
    other = UNetRef(3, 1)
    sd = {k: v.clone() for k, v in other.state_dict().items()}
    nat = UNetNative(3, 1, device=dev, init_from=UNetRef(3, 1))
    tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, plan=True)
    tr.set_batch(x, y)
    for _ in range(4):
        tr.step()
    assert tr.plan_id is not None
    nat.load_state_dict(sd)
    got = [tr.step().clone() for _ in range(3)]
    fresh = UNetNative(3, 1, device=dev, init_from=other)
    tr2 = NativeTrainer(fresh, 2, 64, 64, lr=1e-3, plan=False)
    tr2.set_batch(x, y)
    # tr's Adam moments / step counter continue from the first 4 steps; compare the first loss only
    # (forward of the loaded weights) and that training proceeds on the new weights
    want = tr2.step().clone()
    torch.cuda.synchronize()
    assert torch.equal(got[0][0], want[0])


@pytest.mark.parametrize("plan", [False, True])
def test_overlapped_adam_matches_single_launch_under_stall(plan):
    """NativeAdam's overlapped update (group A on the main stream, group B + re-layouts on the side stream,
    joined by the next forward before down2) is bitwise the single-launch update over several steps; with
    a ~2 ms spin in front of every side-stream Adam launch (eager steps), a forward that read group B's
    weights too early would diverge."""
    from robotic_discovery_platform_amd.models.unet import NativeAdam, UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.ops import native
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(8)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1)
    x = torch.rand(2, 3, 64, 64, device=dev)
    y = (torch.rand(2, 1, 64, 64, device=dev) > 0.5).float()
    C = native()
    orig = C.adam

    def slow(*a, **k):
        if torch.cuda.current_stream() != torch.cuda.default_stream():
            torch.cuda._sleep(5_000_000)
        return orig(*a, **k)
    states = []
    for overlap in (True, False):
        NativeAdam.OVERLAP = overlap
        try:
            if overlap and not plan:
                C.adam = slow
            nat = UNetNative(3, 1, device=dev, init_from=ref)
            tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, plan=plan)
            assert nat._adam_split > 0 and tr._wprep_side() is not None
            tr.set_batch(x, y)
            losses = [tr.step().clone() for _ in range(5)]
            torch.cuda.synchronize()
            states.append((nat.store.flat.clone(), nat.store.shadow.clone(), nat.derived.clone(),
                           nat.store.exp_avg_sq.clone(), int(nat.store.step.item()), torch.stack(losses)))
        finally:
            NativeAdam.OVERLAP = True
            C.adam = orig
    a, b = states
    assert a[4] == b[4] == 5
    for u, v in zip(a[:4] + a[5:], b[:4] + b[5:]):
        assert torch.equal(u, v)


@pytest.mark.parametrize("bilinear", [True, False])
def test_side_stream_wprep_matches_inline(bilinear):
    """NativeTrainer rebuilds the dgrad weight layouts on the wgrad side stream after Adam (overlapping
    the next forward): after every step the derived buffer equals a fresh inline re-layout of the
    masters, the trained state is bitwise that of inline re-layout (graph mode, which keeps it inline),
    and a load_state_dict right after a step waits for the side re-layout."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(6)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1, bilinear=bilinear)
    x = torch.rand(2, 3, 64, 64, device=dev)
    y = (torch.rand(2, 1, 64, 64, device=dev) > 0.5).float()
    nat = UNetNative(3, 1, bilinear=bilinear, device=dev, init_from=ref)
    tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, plan=False)
    assert tr._wprep_side() is not None
    tr.set_batch(x, y)
    for _ in range(3):
        tr.step()
        torch.cuda.synchronize()
        d_side = nat.derived.clone()
        nat.refresh_weights()  # inline re-layout from the same masters
        torch.cuda.synchronize()
        assert torch.equal(d_side, nat.derived)
    nat2 = UNetNative(3, 1, bilinear=bilinear, device=dev, init_from=ref)
    tr2 = NativeTrainer(nat2, 2, 64, 64, lr=1e-3, plan=False)
    tr2._wprep_side = lambda: None  # inline re-layout after Adam
    tr2.set_batch(x, y)
    for _ in range(3):
        tr2.step()
    torch.cuda.synchronize()
    assert torch.equal(nat.store.flat, nat2.store.flat) and torch.equal(nat.derived, nat2.derived)
    sd = {k: v.clone() for k, v in UNetRef(3, 1, bilinear=bilinear).state_dict().items()}
    tr.step()
    nat.load_state_dict(sd)  # right behind the side re-layout of the step
    torch.cuda.synchronize()
    fresh = UNetNative(3, 1, bilinear=bilinear, device=dev, init_from=UNetRef(3, 1, bilinear=bilinear))
    fresh.load_state_dict(sd)
    torch.cuda.synchronize()
    assert torch.equal(nat.derived, fresh.derived)


@pytest.mark.parametrize("h,w", [(64, 96), (224, 224), (48, 80)])
def test_eval_non_power_of_two_widths_match_reference(h, w):
    """Eval (BN folded, row-band convs where the native selector picks them) at map widths that are not
    powers of two: the selector must never pick a kernel the launch rejects (down1 at 64 x 96 has W = 48),
    and every layer it does not pick runs on the implicit GEMM. Compared with UNetRef in eval mode."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(11)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1).to(dev)
    with torch.no_grad():  # non-trivial running statistics
        for name, b in ref.named_buffers():
            if name.endswith("running_mean"):
                b.uniform_(-0.2, 0.2)
            elif name.endswith("running_var"):
                b.uniform_(0.5, 2.0)
    ref.eval()
    nat = UNetNative(3, 1, device=dev, init_from=ref)
    x = torch.rand(1, 3, h, w, device=dev)
    with torch.no_grad():
        want = ref(x.to(torch.bfloat16).float())
    got = nat.forward(x)
    torch.cuda.synchronize()
    assert got.shape == want.shape
    assert _rel(got, want) < 0.08, _rel(got, want)
    ex = nat.executor(1, h, w, training=False)
    from robotic_discovery_platform_amd.ops import native
    C = native()
    for L in ex.layers:  # the executor's fragment copies are exactly the selector's picks
        n_, h_, w_, c1 = L.x1.shape
        c2 = L.x2.shape[3] if L.x2 is not None else 0
        picked = (not L.spec.packed and L.spec.taps == 9
                  and C.rowband_frag_mode(n_, h_, w_, c1, c2, L.spec.cout) > 0)
        assert (L.spec.name in ex._frag_names) == picked, L.spec.name


def test_plan_recorded_after_eval_keeps_adam_joins():
    """An eval (or checkpoint) between steps 2 and 3 clears the overlapped Adam's pending flags; the plan
    recorded at step 3 must still hold the forward's wait on the side-stream update (kind 4) and the
    backward's join of the side stream -- the same op kinds as a plan recorded without the eval."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.ops import native
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(12)
    dev = torch.device("cuda")
    ref = UNetRef(3, 1)
    x = torch.rand(2, 3, 64, 64, device=dev)
    y = (torch.rand(2, 1, 64, 64, device=dev) > 0.5).float()
    C = native()
    kinds, states = [], []
    for interrupt in (False, True):
        nat = UNetNative(3, 1, device=dev, init_from=ref)
        tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, plan=True)
        tr.set_batch(x, y)
        for i in range(5):
            if interrupt and i == 2:
                tr.eval_loss()
                nat.state_dict()
            tr.step()
        torch.cuda.synchronize()
        k = C.plan_kinds(tr.plan_id)
        assert k.count(4) >= 1
        kinds.append(k)
        states.append(nat.store.flat.clone())
    assert kinds[0] == kinds[1]
    assert torch.equal(states[0], states[1])
