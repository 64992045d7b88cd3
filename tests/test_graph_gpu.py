"""The C-ABI kernels are stream-ordered with no host syncs, so CorrBlock (build + lookups), the
warm-start splat and the convex upsampling can be captured into one HIP graph
(torch.cuda.CUDAGraph) and replayed; replay must equal the eager run bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


def _capture(fn):
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()   # warm-up on a side stream, as torch.cuda.graphs recommends
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


@pytest.mark.parametrize("B,H,W", [(1, 32, 32), (4, 60, 80)])
def test_corrblock_graph_replay_bit_exact(ea, B, H, W):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(B * 100 + H)
    f1 = torch.randn((B, 256, H, W), generator=g, device=dev)
    f2 = torch.randn((B, 256, H, W), generator=g, device=dev)
    coords = [(ea.coords_grid(B, H, W, device=dev) + 3 * torch.randn((B, 2, H, W), generator=g, device=dev))
              .contiguous() for _ in range(12)]
    flow = torch.randn((B, 2, H, W), generator=g, device=dev)
    mask = torch.randn((B, 576, H, W), generator=g, device=dev)
    outs = []

    def step():
        outs.clear()
        blk = ea.CorrBlock(f1, f2)
        outs.extend(blk(c) for c in coords)
        outs.append(ea.forward_interpolate_pytorch(flow))
        outs.append(ea.upsample_flow(flow, mask))

    with torch.no_grad():
        step()
        eager = [o.clone() for o in outs]
        graph = _capture(step)
        for c in coords:   # new inputs in place: the replay must see them
            c.add_(0.25)
        graph.replay()
        torch.cuda.synchronize()
        replayed = [o.clone() for o in outs]
        step()
    assert all(torch.equal(a, b) for a, b in zip(replayed, outs))   # replay == eager on the new inputs
    assert not torch.equal(eager[0], replayed[0])
