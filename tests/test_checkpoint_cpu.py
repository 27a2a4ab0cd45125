"""CPU: checkpoint loading of the reference's file layouts with safe loaders only
(model_loader.py:100-177: `net.*` keys, `_extra_state` skipped; wan2pt1.py:648-670 tokenizer.pth)."""
import torch

from cosmos_predict2.checkpoint import load_dit_checkpoint, load_vae_checkpoint
from cosmos_predict2.dit import init_state_dict, state_dict_shapes
from cosmos_predict2.net_config import tiny_dit
from cosmos_predict2.vae import init_vae_state_dict


def test_dit_checkpoint_layouts(tmp_path):
    cfg = tiny_dit(num_blocks=1)
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=0).items()}
    junk = dict(sd)
    junk["net.blocks.0.self_attn.q_proj._extra_state"] = torch.zeros(3)
    junk["net.blocks.0.mlp._extra_state"] = torch.zeros(1)
    # plain dict, and the {"model": ...} wrapper some exporters use
    torch.save(junk, tmp_path / "a.pt")
    torch.save({"model": junk, "step": torch.tensor(7)}, tmp_path / "b.pt")
    for name in ("a.pt", "b.pt"):
        got = load_dit_checkpoint(str(tmp_path / name))
        assert set(got) == set(sd)
        assert all(torch.equal(got[k], sd[k]) for k in sd)
    # every key the net needs is present with the reference's shape
    shapes = state_dict_shapes(cfg)
    assert {k[4:] for k in sd} == set(shapes)
    for k, (shp, dt) in shapes.items():
        assert tuple(sd["net." + k].shape) == tuple(shp), k


def test_safetensors_and_vae(tmp_path):
    from safetensors.torch import save_file

    cfg = tiny_dit(num_blocks=1)
    sd = {"net." + k: v.contiguous() for k, v in init_state_dict(cfg, seed=1).items()}
    save_file(sd, str(tmp_path / "m.safetensors"))
    got = load_dit_checkpoint(str(tmp_path / "m.safetensors"))
    assert set(got) == set(sd) and all(torch.equal(got[k], sd[k]) for k in sd)
    vsd = init_vae_state_dict(seed=0)
    torch.save(vsd, tmp_path / "tokenizer.pth")
    vgot = load_vae_checkpoint(str(tmp_path / "tokenizer.pth"))
    assert set(vgot) == set(vsd)
    assert any(k.startswith("encoder.") for k in vgot) and any(k.startswith("decoder.") for k in vgot)
    assert "conv1.weight" in vgot and "conv2.weight" in vgot
