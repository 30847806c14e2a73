"""bench.py's own multi-rank launch (`--gpus N` with no WORLD_SIZE: the script starts N rank
processes before anything touches a GPU) rehearsed on CPU with `--dry-run` (gloo, the config-4
exchange step at configs[3]'s shape: global batch 256, 32 frames per rank at N = 8, slabs of
capacity(1920, 1080) rows): for N = 1, 2, 4, 8 the line reports n_gpus = N and the matches of
every global frame are identical to the one-rank run; a launcher/--gpus mismatch exits
non-zero."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*argv, env=None):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], cwd=ROOT,
                       env=e, capture_output=True, text=True, timeout=300)
    return p


def _line(p):
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    return json.loads(lines[0])


def test_dry_run_spawns_ranks():
    one = _line(_run("--config", "c4", "--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "1"))
    assert one["n_gpus"] == 1 and one["dry_run"]
    assert one["config"]["global_batch"] == 256
    for n in (2, 4, 8):
        got = _line(_run("--config", "c4", "--gpus", str(n), "--dry-run", "--steps", "2",
                         "--warmup", "1"))
        assert got["n_gpus"] == n
        assert got["config"]["global_batch"] == 256
        assert got["config"]["frames_per_rank_per_step"] == 256 // n
        assert got["match_checksum"] == one["match_checksum"]
        assert got["value"] > 0 and got["steps"] == 2


def test_world_mismatch_fails():
    p = _run("--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0",
             env={"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
    assert "--gpus 2" in p.stderr
