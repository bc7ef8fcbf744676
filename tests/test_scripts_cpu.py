"""Golden-output tests for the reference-compatible CLIs (survey §4 item 7, Appendix B): the
toy all-reduce script and the MNIST trainer on the CPU/gloo path, launched both the reference way
(one process per rank with -i/-r/-s) and through the framework launcher."""
import json
import os
import re
import subprocess
import sys

import pytest

from pytorch_distributed_example_amd.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONWARNINGS="ignore::FutureWarning", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
TOY_LINE = re.compile(r"^rank: (\d+), step: (\d+), value: (\d+), reduced sum: ([0-9.]+)\.$")
EPOCH_LINE = re.compile(r"^Epoch: (\d+)/(\d+), train loss: ([0-9.]+), train acc: ([0-9.]+)%, "
                        r"test loss: ([0-9.]+), test acc: ([0-9.]+)%?\.$")


def _check_toy(lines, world, steps):
    rows = [TOY_LINE.match(l) for l in lines]
    rows = [tuple(map(float, m.groups())) for m in rows if m]
    assert len(rows) == world * steps
    for step in range(1, steps + 1):
        at = [r for r in rows if r[1] == step]
        assert sorted(int(r[0]) for r in at) == list(range(world))
        assert len({r[3] for r in at}) == 1                     # every rank printed the same sum
        assert at[0][3] == sum(r[2] for r in at)


def test_toy_reference_style_three_shells():
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "scripts/toy.py"), "-i", f"tcp://127.0.0.1:{port}",
                               "-r", str(r), "-s", "3", "--steps", "4", "--sleep", "0"], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True, env=ENV) for r in range(3)]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert outs[0].splitlines()[0].startswith("Namespace(backend='gloo', init_method=")
    _check_toy([l for o in outs for l in o.splitlines()], 3, 4)


def test_toy_via_launcher():
    out = subprocess.run([sys.executable, "-m", "pytorch_distributed_example_amd.launch", "-n", "4",
                          os.path.join(ROOT, "scripts/toy.py"), "--steps", "3", "--sleep", "0"], cwd=ROOT,
                         capture_output=True, text=True, env=ENV, timeout=180)
    assert out.returncode == 0, out.stderr
    _check_toy(out.stdout.splitlines(), 4, 3)


def _mnist(args, n=None, timeout=300):
    base = [os.path.join(ROOT, "scripts/mnist.py"), "--no-cuda", "--train-size", "1024", "--test-size", "256",
            "--epochs", "2"] + args
    if "--cprofile" not in args:
        base.append("--no-cprofile")          # the default (reference parity) writes ./stats
    cmd = [sys.executable] + (["-m", "pytorch_distributed_example_amd.launch", "-n", str(n)] if n else []) + base
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, env=ENV, timeout=timeout)
    assert out.returncode == 0, out.stdout + out.stderr
    return out.stdout.splitlines()


def test_mnist_single_process_golden():
    lines = _mnist(["-s", "1"])
    assert lines[0].startswith("Namespace(backend='nccl', init_method='tcp://127.0.0.1:23456', rank=None, "
                               "world_size=1, epochs=2, no_cuda=True, learning_rate=0.001, root='data', "
                               "batch_size=128, eval=False")
    assert "bucket_mb=25.0, dtype='fp32'" in lines[0]              # additive flags and defaults
    assert lines[1:4] == ["device = cpu", "Getting data loader with root = data", "obtained data_loader"]
    ep = [EPOCH_LINE.match(l) for l in lines[4:]]
    assert all(ep) and len(ep) == 2
    assert ep[0].group(5) == "0" and ep[0].group(6) == "0"      # no --eval: zeros until the last epoch
    assert float(ep[1].group(3)) < float(ep[0].group(3))         # loss decreases


@pytest.mark.parametrize("ddp", ["on", "off"])
def test_mnist_gloo_two_ranks(ddp):
    lines = _mnist(["--backend", "gloo", "--eval", "--ddp", ddp], n=2)
    assert lines.count("called init_process_group") == 2
    ep = [m for m in map(EPOCH_LINE.match, lines) if m]
    assert len(ep) == 4
    # test metrics identical across ranks (replicas in sync)
    last = [m for m in ep if m.group(1) == "2"]
    assert last[0].group(5) == last[1].group(5) and last[0].group(6) == last[1].group(6)


def test_mnist_bucket_mb_reaches_ddp():
    """--bucket-mb re-cuts DDP's gradient buckets: 0.05 MB splits the toy CNN's 1.72 MB of gradients into
    several buckets (fc1.weight alone is 1.6 MB), and the replicas' printed metrics are identical to the
    default single-bucket run (a bucket boundary does not change the elementwise 2-rank sum)."""
    from pytorch_distributed_example_amd.models import build_net
    from pytorch_distributed_example_amd.parallel.ddp import reverse_order_buckets
    shapes = [(n, tuple(p.shape)) for n, p in build_net(seed=0).named_parameters()]
    assert len(reverse_order_buckets(shapes, int(0.05 * (1 << 20)), 4)) > 2
    assert len(reverse_order_buckets(shapes, int(25.0 * (1 << 20)), 4)) == 1
    common = ["--backend", "gloo", "--eval", "--epochs", "1", "--log-rank0-only"]
    small = [l for l in _mnist(common + ["--bucket-mb", "0.05"], n=2) if EPOCH_LINE.match(l)]
    default = [l for l in _mnist(common, n=2) if EPOCH_LINE.match(l)]
    assert small == default and len(small) == 1


def test_mnist_dtype_bf16_autocast():
    """--dtype bf16: the forward runs under torch.autocast (bf16 matmuls / convs) with fp32 parameters and
    optimizer state; it trains (loss decreases) and differs from the fp32 run (bf16 is really in use)."""
    lines = _mnist(["-s", "1", "--dtype", "bf16", "--epochs", "2"])
    assert "dtype='bf16'" in lines[0]
    ep = [m for m in map(EPOCH_LINE.match, lines) if m]
    assert len(ep) == 2 and float(ep[1].group(3)) < float(ep[0].group(3))
    fp = [m for m in map(EPOCH_LINE.match, _mnist(["-s", "1", "--epochs", "2"])) if m]
    assert ep[0].group(3) != fp[0].group(3)


def test_config1_mlp_gloo_two_ranks(tmp_path):
    """BASELINE.json config 1: 2-layer MLP, gloo (host TCP) backend, world_size 2, CPU only."""
    metrics = str(tmp_path / "m.jsonl")
    lines = _mnist(["--backend", "gloo", "--eval", "--model", "mlp", "--epochs", "3", "--metrics", metrics], n=2)
    assert lines.count("called init_process_group") == 2
    ep = [m for m in map(EPOCH_LINE.match, lines) if m]
    assert len(ep) == 6
    by_rank_epoch = {}
    for m in ep:
        by_rank_epoch.setdefault(m.group(1), []).append(m)
    # replicas identical: every epoch's full-test-set loss / accuracy agree to the printed digit
    for e, ms in by_rank_epoch.items():
        assert len(ms) == 2 and ms[0].group(5) == ms[1].group(5) and ms[0].group(6) == ms[1].group(6), e
    train = [float(by_rank_epoch[str(e)][0].group(3)) for e in (1, 2, 3)]
    assert train[2] < train[1] < train[0], train                 # loss decreases
    recs = [json.loads(l) for l in open(metrics)]
    assert len(recs) == 3 and all(r["images_per_s"] > 0 for r in recs)


def test_mnist_save_resume(tmp_path):
    ck = str(tmp_path / "ck.pt")
    _mnist(["-s", "1", "--save", ck, "--epochs", "1"])
    assert os.path.exists(ck)
    lines = _mnist(["-s", "1", "--resume", ck, "--epochs", "2"])
    ep = [m for m in map(EPOCH_LINE.match, lines) if m]
    assert [m.group(1) for m in ep] == ["2"]


def test_resume_set_epoch_matches_uninterrupted(tmp_path):
    """--resume continues the sampler's epoch numbering: with --set-epoch, epochs 1+2 in
    one run print the same epoch-2 line as epoch 1, save, resume, epoch 2."""
    ck = str(tmp_path / "ck.pt")
    common = ["--backend", "gloo", "--set-epoch", "--model", "mlp", "--log-rank0-only"]
    full = [m for m in map(EPOCH_LINE.match, _mnist(common + ["--epochs", "2"], n=2)) if m]
    _mnist(common + ["--epochs", "1", "--save", ck], n=2)
    res = [m for m in map(EPOCH_LINE.match, _mnist(common + ["--epochs", "2", "--resume", ck], n=2)) if m]
    assert [m.group(1) for m in res] == ["2"]
    assert res[0].group(0) == full[1].group(0)


def test_read_stats(tmp_path):
    prof = str(tmp_path / "p.prof")
    _mnist(["-s", "1", "--epochs", "1", "--cprofile", prof])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts/read_stats.py"), prof, "10"],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "tottime" in out.stdout and "internal time" in out.stdout
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts/read_stats.py"), prof, "5", "--sort",
                          "cumulative"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "cumulative time" in out.stdout


def test_toy_via_torchrun():
    """The driver's multi-GPU launcher path: torch.distributed.run owns MASTER_PORT (agent store)."""
    port = free_port()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "scripts/toy.py"), "--steps", "2", "--sleep", "0"], cwd=ROOT,
                         capture_output=True, text=True, env=ENV, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.replace("rank:", "\nrank:").splitlines() if l.startswith("rank:")]
    _check_toy(lines, 3, 2)
