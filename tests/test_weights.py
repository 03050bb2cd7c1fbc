"""Checkpoint loading (arbius_amd/models/weights.py): diffusers/transformers names -> the engine's
fused / channels-last modules.  The CLIP mapping is checked against transformers' own
CLIPTextModel (numerical parity of the encoder, not just the names); the UNet / VAE mapping by a
diffusers-layout export -> load round trip (diffusers itself is not installed here)."""
import os

import pytest
import torch

from arbius_amd.models import weights as W
from arbius_amd.models.clip_text import CLIPTextConfig, CLIPTextEncoder
from arbius_amd.models.registry import build_pipeline


@pytest.mark.parametrize("act", ["quick_gelu", "gelu"])   # ViT-L/14 (SD1.5, Kandinsky prior) / ViT-H/14 (zeroscope)
def test_clip_text_matches_transformers_clip(act):
    transformers = pytest.importorskip("transformers")
    torch.manual_seed(0)
    hf_cfg = transformers.CLIPTextConfig(vocab_size=1000, hidden_size=64, intermediate_size=128,
                                         num_hidden_layers=2, num_attention_heads=4, max_position_embeddings=77,
                                         hidden_act=act, bos_token_id=0, eos_token_id=2)
    hf = transformers.CLIPTextModel(hf_cfg).eval()
    ours = CLIPTextEncoder(CLIPTextConfig(vocab=1000, max_len=77, width=64, layers=2, heads=4, mlp=128,
                                          quick_gelu=act == "quick_gelu")).eval()
    src = W.normalize_clip_names(dict(hf.state_dict()))
    W.load_state(ours, W.convert(W.RULES["text"](), dict(ours.named_parameters()), src))
    ids = torch.randint(1, 998, (2, 77))
    ids[:, 10] = 999                                   # EOS = the largest id (pooled-token rule)
    with torch.no_grad():
        ref = hf(input_ids=ids).last_hidden_state
        got, _ = ours(ids)
    assert torch.allclose(got, ref, atol=2e-5, rtol=1e-4), (got - ref).abs().max()


def _params(pipe):
    return {f"{m}.{k}": v.detach().clone() for m, mod in pipe.modules().items() for k, v in mod.named_parameters()}


def test_sd15_diffusers_layout_round_trip(tmp_path):
    a = build_pipeline("anythingv3", tiny=True, weight_seed=0)
    for name, state in W.export_diffusers(a).items():
        W.write_safetensors(state, os.path.join(tmp_path, W._DIFFUSERS[name]))
    # the exported names are the public ones
    unet = W.read_safetensors(os.path.join(tmp_path, W._DIFFUSERS["unet"]))
    assert "down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q.weight" in unet
    assert unet["conv_in.weight"].shape[1] == 4                                   # OIHW on disk
    b = build_pipeline("anythingv3", tiny=True, weight_seed=7, weights_dir=str(tmp_path))
    pa, pb = _params(a), _params(b)
    assert pa.keys() == pb.keys() and all(torch.equal(pa[k], pb[k]) for k in pa)


def test_native_layout_round_trip_and_strictness(tmp_path):
    a = build_pipeline("anythingv3", tiny=True, weight_seed=1)
    W.save_native(a, str(tmp_path))
    b = build_pipeline("anythingv3", tiny=True, weight_seed=2, weights_dir=str(tmp_path))
    pa, pb = _params(a), _params(b)
    assert all(torch.equal(pa[k], pb[k]) for k in pa)
    # a checkpoint that misses a tensor must fail loudly, never half-load
    st = W.read_safetensors(os.path.join(tmp_path, "unet.safetensors"))
    st.pop("conv_in.weight")
    W.write_safetensors(st, os.path.join(tmp_path, "unet.safetensors"))
    with pytest.raises(KeyError):
        build_pipeline("anythingv3", tiny=True, weights_dir=str(tmp_path))


def test_missing_weights_dir_is_an_error(tmp_path):
    with pytest.raises(FileNotFoundError):
        build_pipeline("anythingv3", tiny=True, weights_dir=str(tmp_path))


def test_mclip_xlmr_matches_transformers_xlm_roberta():
    """Kandinsky's multilingual text tower (post-LN XLM-R, per-sequence K/V slicing instead of a
    key mask) == transformers XLMRobertaModel with an attention mask, pads included."""
    transformers = pytest.importorskip("transformers")
    from arbius_amd.models.xlmr import MCLIPText, XLMRConfig
    torch.manual_seed(0)
    hf_cfg = transformers.XLMRobertaConfig(vocab_size=1000, hidden_size=32, num_hidden_layers=2,
                                           num_attention_heads=2, intermediate_size=64, max_position_embeddings=100,
                                           type_vocab_size=1, pad_token_id=1, layer_norm_eps=1e-5)
    hf = transformers.XLMRobertaModel(hf_cfg, add_pooling_layer=False).eval()
    ours = MCLIPText(XLMRConfig.tiny()).eval()
    src = {"transformer." + k: v for k, v in hf.state_dict().items()}
    src["LinearTransformation.weight"] = torch.randn(32, 32)
    src["LinearTransformation.bias"] = torch.randn(32)
    target = dict(ours.named_parameters())
    W.load_state(ours, W.convert(W.RULES["mclip"](), target, src))
    n = 9
    ids = torch.full((1, 77), 1, dtype=torch.long)
    ids[0, :n] = torch.randint(3, 999, (n,))
    ids[0, 0], ids[0, n - 1] = 0, 2
    mask = (ids != 1).long()
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).last_hidden_state
        got, pooled = ours(ids, n)
    assert torch.allclose(got, ref, atol=3e-5, rtol=1e-4), (got - ref).abs().max()
    exp_pool = ref[:, :n].mean(1) @ src["LinearTransformation.weight"].T + src["LinearTransformation.bias"]
    assert torch.allclose(pooled, exp_pool, atol=3e-5, rtol=1e-4)
