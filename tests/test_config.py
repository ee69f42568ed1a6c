"""Config system: presets (XOR semantics, reference D8), aliases (D14), YAML + overrides, CfgNode."""
import os
import pytest

from mingpt_distributed_amd.models.config import GPTConfig, PRESETS
from mingpt_distributed_amd.utils.config import CfgNode, load_run_config


def test_preset_only():
    c = GPTConfig(model_type="gpt-nano", vocab_size=3, block_size=11).resolve()
    assert (c.n_layer, c.n_head, c.n_embed) == (3, 3, 48)


def test_explicit_dims_win_over_default_model_type():
    # the reference YAML gives dims while GPTConfig.model_type defaults to "gpt2" (D8)
    c = GPTConfig(n_layer=8, n_head=8, n_embd=512).resolve()
    assert (c.n_layer, c.n_head, c.n_embed) == (8, 8, 512)


def test_partial_dims_rejected():
    with pytest.raises(ValueError):
        GPTConfig(n_layer=2).resolve()


def test_bad_head_split():
    with pytest.raises(ValueError):
        GPTConfig(n_layer=2, n_head=5, n_embed=48).resolve()


def test_aliases():
    c = GPTConfig(n_layer=1, n_head=1, n_embd=8, embd_pdrop=0.2, resid_pdrop=0.3, attn_pdrop=0.4)
    assert c.n_embed == 8 and c.embed_drop == 0.2 and c.resid_drop == 0.3 and c.attn_drop == 0.4
    assert c.n_embd == 8 and c.attn_pdrop == 0.4
    with pytest.raises(TypeError):
        GPTConfig(bogus=1)


def test_presets_table():
    assert PRESETS["gpt2-xl"] == dict(n_layer=48, n_head=25, n_embed=1600)
    assert set(PRESETS) >= {"openai-gpt", "gpt2", "gpt2-medium", "gpt2-large", "gpt2-xl", "gopher-44m",
                            "gpt-mini", "gpt-micro", "gpt-nano"}


def test_cfgnode_merge():
    C = CfgNode(a=1, sub=CfgNode(b=2.0, c="x"))
    C.merge_from_args(["--sub.b=3.5", "a=7", "--sub.c=hello"])
    assert C.a == 7 and C.sub.b == 3.5 and C.sub.c == "hello"
    with pytest.raises(AssertionError):
        C.merge_from_args(["--sub.nope=1"])
    C.merge_from_dict({"sub": {"b": 1}})
    assert C.sub.b == 1
    assert "sub:" in str(C)
    assert C.to_dict() == {"a": 7, "sub": {"b": 1, "c": "hello"}}


def test_reference_yaml_shape(tmp_path):
    y = tmp_path / "cfg.yaml"
    y.write_text("""
gpt_config: {n_layer: 8, n_head: 8, n_embd: 512}
optimizer_config: {weight_decay: 0.1, learning_rate: 0.0003}
data_config: {path: s3://bucket, block_size: 128, truncate: 0.05}
trainer_config: {max_epochs: 10, batch_size: 64, dl_num_workers: 4, grad_norm_clip: 1.0,
                 snapshot_path: s3://bucket/gpt_snapshot.pt, save_every: 3}
hydra: {run: {dir: ./}}
""")
    rc = load_run_config(str(y), ["trainer_config.batch_size=32", "--optimizer_config.learning_rate=1e-3"])
    assert rc.gpt_config.n_embed == 512
    assert rc.trainer_config.batch_size == 32
    assert rc.optimizer_config.learning_rate == 1e-3
    assert rc.data_config.train_split == 0.9  # D13: default when the YAML omits it
    with pytest.raises(KeyError):
        load_run_config(str(y), ["gpt_config.nonsense=1"])


def test_zero1_override_reaches_trainer_config():
    from mingpt_distributed_amd.utils.config import load_run_config

    assert load_run_config(None, ["trainer_config.zero1=true"]).trainer_config.zero1 is True
    assert load_run_config(None, []).trainer_config.zero1 is False


def test_bench_refuses_more_gpus_than_visible():
    """`bench.py --gpus N` without a torchrun env launches N ranks itself, and fails loudly (never
    a silent 1-GPU number labelled N) when fewer GPUs are visible -- here, on CPU, zero are."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 2 requested but only 0 GPU(s) are visible" in r.stderr
