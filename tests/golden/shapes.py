"""State-dict (name, shape) lists of the reference modules, so tests can rebuild the seeded
weights without importing the reference (`model.py:496-529`, `network.py:23-30,115-117`)."""

TOY = dict(dim=256, ffn_dim=512, freq_dim=256, text_dim=64, num_heads=2, num_layers=2,
           out_dim=16, text_len=512)
REAL = dict(dim=5120, ffn_dim=13824, freq_dim=256, text_dim=4096, num_heads=40, num_layers=40,
            out_dim=16, text_len=512)


def block_shapes(prefix, dim, ffn, i2v=False):
    s = [(prefix + "modulation", (1, 6, dim))]
    for att in ("self_attn", "cross_attn"):
        for p in ("q", "k", "v", "o"):
            s += [(f"{prefix}{att}.{p}.weight", (dim, dim)), (f"{prefix}{att}.{p}.bias", (dim,))]
        s += [(f"{prefix}{att}.norm_q.weight", (dim,)), (f"{prefix}{att}.norm_k.weight", (dim,))]
    if i2v:
        for p in ("k_img", "v_img"):
            s += [(f"{prefix}cross_attn.{p}.weight", (dim, dim)),
                  (f"{prefix}cross_attn.{p}.bias", (dim,))]
        s += [(f"{prefix}cross_attn.norm_k_img.weight", (dim,))]
    s += [(prefix + "norm3.weight", (dim,)), (prefix + "norm3.bias", (dim,)),
          (prefix + "ffn.0.weight", (ffn, dim)), (prefix + "ffn.0.bias", (ffn,)),
          (prefix + "ffn.2.weight", (dim, ffn)), (prefix + "ffn.2.bias", (dim,))]
    return s


def model_shapes(cfg, model_type="t2v", num_layers=None, head=True):
    d, f = cfg["dim"], cfg["ffn_dim"]
    in_dim = 16 if model_type == "t2v" else 36
    s = [("patch_embedding.weight", (d, in_dim, 1, 2, 2)), ("patch_embedding.bias", (d,)),
         ("text_embedding.0.weight", (d, cfg["text_dim"])), ("text_embedding.0.bias", (d,)),
         ("text_embedding.2.weight", (d, d)), ("text_embedding.2.bias", (d,)),
         ("time_embedding.0.weight", (d, cfg["freq_dim"])), ("time_embedding.0.bias", (d,)),
         ("time_embedding.2.weight", (d, d)), ("time_embedding.2.bias", (d,)),
         ("time_projection.1.weight", (6 * d, d)), ("time_projection.1.bias", (6 * d,))]
    for i in range(cfg["num_layers"] if num_layers is None else num_layers):
        s += block_shapes(f"blocks.{i}.", d, f, model_type != "t2v")
    if head:
        s += [("head.head.weight", (4 * cfg["out_dim"], d)), ("head.head.bias", (4 * cfg["out_dim"],)),
              ("head.modulation", (1, 2, d))]
    if model_type != "t2v":
        s += [("img_emb.proj.0.weight", (1280,)), ("img_emb.proj.0.bias", (1280,)),
              ("img_emb.proj.1.weight", (1280, 1280)), ("img_emb.proj.1.bias", (1280,)),
              ("img_emb.proj.3.weight", (d, 1280)), ("img_emb.proj.3.bias", (d,)),
              ("img_emb.proj.4.weight", (d,)), ("img_emb.proj.4.bias", (d,))]
    return s


def qa_shapes(E):
    return [("queries", (1, E)), ("multihead_attn.in_proj_weight", (3 * E, E)),
            ("multihead_attn.in_proj_bias", (3 * E,)), ("multihead_attn.out_proj.weight", (E, E)),
            ("multihead_attn.out_proj.bias", (E,))]


def mlp_shapes(E):
    return [("fc1.weight", (1024, E)), ("fc1.bias", (1024,)), ("fc2.weight", (512, 1024)),
            ("fc2.bias", (512,)), ("fc3.weight", (1, 512)), ("fc3.bias", (1,))]


def seeded_params(shapes, prefix="", seed=None):
    """{name: torch fp32 tensor} with the same draw make_golden.py loaded into the reference."""
    import torch
    import seeded
    seed = seeded.BASE_SEED if seed is None else seed
    return {n: torch.from_numpy(seeded.make_param(prefix + n, s, seed)) for n, s in shapes}
