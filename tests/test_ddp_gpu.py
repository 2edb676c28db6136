"""The distributed train step on the HIP engine (basicsr/models/base_model.py:87-105 DDP
semantics): two ranks (gloo, both on cuda:0 -- the GPU box has one device) each train on half
of a batch; the bucketed all-reduce launched from the HIP gradient-ready callbacks plus the
1/world scale folded into the fused Adam must reproduce single-process training on the full
batch.  fp32 parity mode, 2 steps, relative 2e-4."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _collect(q, procs, n, timeout=240):
    """n results from the worker queue; fails fast (instead of waiting out the timeout) when a
    worker dies, and prints a heartbeat so a slow run is not mistaken for a hang."""
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < n:
        try:
            out.append(q.get(timeout=10))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f'worker died: exit codes {dead}'
            assert time.time() - t0 < timeout, 'workers timed out'
            print(f'  waiting for workers ({time.time() - t0:.0f} s)', flush=True)
    return out


EDSR_S = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, upscale=4, res_scale=1)
RCAN_S = dict(type='RCAN', num_in_ch=3, num_out_ch=3, num_feat=64, num_group=2, num_block=2, squeeze_factor=16,
              upscale=4, res_scale=1)


def _opt(dist_, world, rank, bucket_mb, async_wgrad=False, graph=False, net=EDSR_S):
    return dict(model_type='SRModel', is_train=True, dist=dist_, num_gpu=1, world_size=world, rank=rank, path={},
                bucket_cap_mb=bucket_mb,
                network_g=dict(net),
                train=dict(ema_decay=0.999, use_amp=False, async_wgrad=async_wgrad, cuda_graph=graph,
                           optim_g=dict(type='Adam', lr=1e-3, weight_decay=0, betas=[0.9, 0.99]),
                           scheduler=dict(type='MultiStepLR', milestones=[100], gamma=0.5),
                           pixel_opt=dict(type='L1Loss', loss_weight=1.0, reduction='mean')))


def _batch(step):
    g = torch.Generator().manual_seed(50 + step)
    return torch.rand(4, 3, 16, 16, generator=g), torch.rand(4, 3, 64, 64, generator=g)


def _worker(rank, world, port, bucket_mb, async_wgrad, q, graph=False, steps=2):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    if async_wgrad:
        # two ranks share the one card, where SRModel turns the side stream off;
        # SR_ASYNC_WGRAD=1 keeps it on so this test covers DDP + side streams (eager steps only)
        os.environ['SR_ASYNC_WGRAD'] = '1'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    torch.manual_seed(0 + rank)  # different init per rank: the reducer broadcasts rank 0's
    model = build_model(_opt(True, world, rank, bucket_mb, async_wgrad, graph))
    assert bool(model.async_wgrad) == bool(async_wgrad), 'side-stream mode silently changed'
    for step in range(1, steps + 1):
        lq, gt = _batch(step)
        sl = slice(rank * 2, rank * 2 + 2)
        model.feed_data({'lq': lq[sl], 'gt': gt[sl]})
        model.update_learning_rate(step)
        model.optimize_parameters(step)
    net = model.get_bare_model(model.net_g)
    sd = {k: v.detach().cpu().numpy().copy() for k, v in net.state_dict().items()}  # by value, not fd-shared
    red = model.net_g.reducer
    nseg = model._graph.n_segments if graph else 0
    q.put((rank, sd, len(red.buckets), list(red.last_issue_log), nseg))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('async_wgrad', [False, True])
@pytest.mark.parametrize('bucket_mb', [25.0, 0.05])
def test_ddp_two_ranks_match_full_batch(cuda, bucket_mb, async_wgrad):
    """async_wgrad: weight gradients on the side stream, buckets issued from it (utils/flat.py)."""
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bucket_mb, async_wgrad, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for rank, sd, nb, log, _ in _collect(q, procs, 2):
        res[rank] = (sd, nb, log)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if bucket_mb < 1:
        assert res[0][1] > 1  # several buckets
    # every bucket's all-reduce was issued from a gradient-ready callback while backward was
    # still running (overlap), none only at the join before the optimizer; same order on both ranks
    for r in (0, 1):
        log = res[r][2]
        assert sorted(b for b, _ in log) == list(range(res[r][1])), log
        assert all(when == 'backward' for _, when in log), log
    assert res[0][2] == res[1][2]
    # both ranks hold identical parameters
    for k in res[0][0]:
        assert (res[0][0][k] == res[1][0][k]).all(), k
    # and they equal single-process training on the whole batch from rank 0's init
    torch.manual_seed(0)
    ref = build_model(_opt(False, 1, 0, bucket_mb))
    for step in (1, 2):
        lq, gt = _batch(step)
        ref.feed_data({'lq': lq, 'gt': gt})
        ref.update_learning_rate(step)
        ref.optimize_parameters(step)
    for k, v in ref.get_bare_model(ref.net_g).state_dict().items():
        got = torch.from_numpy(res[0][0][k])
        err = (got - v.cpu()).abs().max().item() / max(1e-3, v.abs().max().item())
        assert err < 2e-4, (k, err)


def test_ddp_graph_segments_match_full_batch(cuda, async_wgrad=False):
    """train.cuda_graph with DDP: steps 1-2 eager, step 3 captured as graph segments cut at the ready
    buckets (utils/step_graph.py), steps 4-5 replayed with the bucket all-reduces launched between
    segments.  Two gloo ranks on the one card, fp32: both ranks equal, and equal to single-process
    eager training on the full batch (relative 2e-4); every bucket but the flushed tail goes out
    between backward segments.  (Side streams under the segmented graph: the RCCL world-1 tests
    below, where one process owns the card.)"""
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 0.05, async_wgrad, q, True, 5)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for rank, sd, nb, log, nseg in _collect(q, procs, 2):
        res[rank] = (sd, nb, log, nseg)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nb = res[0][1]
    assert nb > 1
    for r in (0, 1):
        log, nseg = res[r][2], res[r][3]
        assert sorted(b for b, _ in log) == list(range(nb)), log
        assert sum(1 for _, w in log if w == 'backward') >= nb - 1, log
        assert nseg >= 3, nseg
    assert res[0][2] == res[1][2]
    for k in res[0][0]:
        assert (res[0][0][k] == res[1][0][k]).all(), k
    torch.manual_seed(0)
    ref = build_model(_opt(False, 1, 0, 0.05))
    for step in range(1, 6):
        lq, gt = _batch(step)
        ref.feed_data({'lq': lq, 'gt': gt})
        ref.update_learning_rate(step)
        ref.optimize_parameters(step)
    for k, v in ref.get_bare_model(ref.net_g).state_dict().items():
        got = torch.from_numpy(res[0][0][k])
        err = (got - v.cpu()).abs().max().item() / max(1e-3, v.abs().max().item())
        assert err < 2e-4, (k, err)


def _nccl_worker(port, q, async_wgrad=False, netcfg=EDSR_S):
    """World 1 over RCCL: the segmented graph's replay issues real RCCL all-reduces."""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1)
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    out = []
    for graph in (False, True):
        torch.manual_seed(0)
        o = _opt(True, 1, 0, 0.05, async_wgrad, graph, netcfg)
        o['train']['use_amp'] = True
        model = build_model(o)
        assert bool(model.async_wgrad) == bool(async_wgrad), 'side-stream mode silently changed'
        if async_wgrad:
            red = model.net_g.reducer
            assert len(red.buckets) > 4  # 50 KB buckets: gradient-ready callbacks cut inside a block's fork
        if graph:
            # hold each capture for a while so RCCL's watchdog thread polls its pending work (an event
            # query) during it: in the global capture mode that poll aborts the process
            import time

            def _slow_capture(mod, inp):
                if torch.cuda.is_current_stream_capturing():
                    time.sleep(0.3)
            model.get_bare_model(model.net_g).register_forward_pre_hook(_slow_capture)
        losses = []
        for step in range(1, 6):
            lq, gt = _batch(step)
            model.feed_data({'lq': lq, 'gt': gt})
            model.update_learning_rate(step)
            if graph and step == 3:  # the capture step: a collective still in the watchdog's list
                dist.all_reduce(torch.ones(1, device='cuda'))
            model.optimize_parameters(step)
            losses.append(model.get_current_log()['l_pix'])
        net = model.get_bare_model(model.net_g)
        out.append((losses, {k: v.detach().cpu().numpy().copy() for k, v in net.state_dict().items()},
                    model._graph.n_segments if graph else 0))
    dist.destroy_process_group()
    q.put(out)


def test_ddp_graph_segments_rccl_world1_bitwise(cuda):
    """The segmented-graph DDP step over RCCL (world 1 on the one card, bf16): graph replays are
    bitwise equal to the eager DDP steps, and a capture that overlaps a poll of RCCL's watchdog
    thread survives it (thread-local capture mode; round 4: `bench.py --ddp` aborted in global mode)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    ((l0, s0, _), (l1, s1, nseg)), = _collect(q, [p], 1)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert nseg >= 3
    assert l0 == l1
    for k in s0:
        assert (s0[k] == s1[k]).all(), k


@pytest.mark.parametrize('net', ['edsr', 'rcan'])
def test_ddp_graph_segments_async_rccl_world1_bitwise(cuda, net):
    """Side-stream weight gradients (train.async_wgrad, forks batched per block) under the segmented
    DDP graph over RCCL, with 50 KB buckets so a gradient-ready callback completes a bucket -- and
    cuts the capture -- in the middle of a block's batched fork: every launch of the fork must be
    inside the graph, so the replayed steps equal the eager ones bitwise (a launch left out of the
    graph would leave its weight gradient stale at replay)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q, True, EDSR_S if net == 'edsr' else RCAN_S))
    p.start()
    ((l0, s0, _), (l1, s1, nseg)), = _collect(q, [p], 1)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert nseg >= 3
    assert l0 == l1
    for k in s0:
        assert (s0[k] == s1[k]).all(), k
