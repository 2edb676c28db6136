"""bench.py's launch contract on the CPU (no GPU): ``--gpus N`` must run N ranks.

``python bench.py --gpus 2`` started without a launcher spawns torch.distributed.run with two rank
processes; the rank-0 line reports ``n_gpus: 2`` and ``dp2`` and the max-over-ranks timing ran
over both (``--dry-run``: gloo rendezvous, barriers and the MAX all-reduce with a no-op step).  A
launcher WORLD_SIZE that disagrees with ``--gpus`` exits non-zero.  Reference launch:
scripts/dist_train.sh:7 (torch.distributed.launch --nproc_per_node)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def _line(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, (p.stdout, p.stderr)
    return json.loads(lines[0])


def test_bench_gpus2_spawns_two_ranks():
    p = _run(['--gpus', '2', '--dry-run', '--steps', '3', '--workload', 'rcan'])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p)
    assert d['n_gpus'] == 2 and d['ranks_seen'] == 2
    assert d['config']['parallelism'] == 'dp2'
    assert d['config']['global_batch'] == 2 * d['config']['per_gpu_batch'] == 64
    assert d['config']['hip_graph'] is True


def test_bench_gpus1_single_process():
    p = _run(['--dry-run', '--steps', '2', '--workload', 'edsr'])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p)
    assert d['n_gpus'] == 1 and d['config']['parallelism'] == 'dp1'


def test_bench_world_size_mismatch_fails():
    p = _run(['--gpus', '4', '--dry-run'], env_extra={'WORLD_SIZE': '2', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert p.returncode != 0
    assert 'disagrees with WORLD_SIZE' in p.stderr


def test_pmc_traffic_record_per_dominant_kernel():
    """bench.py's roofline.traffic comes from profiles/pmc_traffic.json: the record of the workload
    whose bench kernel is the dominant one, also an extra record of that workload ('<wl>_<what>')
    when a close contender dominates (SwinIR: linear_wk_kernel / linear_wgrad_kernel+reduce)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for wl, kernel in (('edsr', 'conv3x3_fwd_pph_kernel'), ('swinir', 'linear_wk_kernel'),
                       ('swinir', 'linear_wgrad_kernel+reduce'), ('rcan', 'conv3x3_fwd_band_kernel')):
        rec = bench._pmc_traffic(wl, kernel)
        assert rec is not None and rec['bench_kernel'] == kernel and rec['hbm_bytes_per_launch'] > 0, (wl, kernel)
    assert bench._pmc_traffic('edsr', 'linear_wk_kernel') is None  # another workload's record never answers


def test_bench_suite_sub_records_per_workload():
    """A plain N = 1 run measures the EDSR headline and RCAN / SwinIR / RRDB each in a child
    process (the parent never touches the GPU) and prints ONE line: the headline's fields, then
    ``workloads`` as the last key (the driver keeps the tail of stdout) with one compact record per
    BASELINE config."""
    p = _run(['--dry-run', '--steps', '2'])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p)
    assert d['config']['model'] == 'EDSR' and d['config']['baseline_config'] == 'configs[1]'
    assert d['suite']['parent_touches_gpu'] is False
    assert list(d)[-1] == 'workloads'
    assert list(d['workloads']) == ['edsr', 'rcan', 'swinir', 'rrdb']
    cfg = {wl: r['config'] for wl, r in d['workloads'].items()}
    assert cfg == {'edsr': 'configs[1]', 'rcan': 'configs[2]', 'swinir': 'configs[3]', 'rrdb': 'configs[4]'}
    for wl, r in d['workloads'].items():
        assert r['rc'] == 0 and 'roofline' in r and 'cpu_baseline' in r and 'parity' in r, (wl, r)
    assert set(d['sub_records']) == {'rcan', 'swinir', 'rrdb'}
    assert d['sub_records']['rrdb']['config']['per_gpu_batch'] == 16


def test_bench_lr_px_sweep_label():
    """--lr-px (SURVEY §8 secondary sweep, LR 256 -> HR 1024) changes the tile in the label."""
    p = _run(['--dry-run', '--steps', '1', '--workload', 'swinir', '--lr-px', '256', '--batch', '2'])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p)
    assert d['config']['lr_tile'] == 256 and 'LR 256x256 -> HR 1024x1024' in d['config']['workload']
    assert d['config']['per_gpu_batch'] == 2
