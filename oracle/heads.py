"""CPU oracle for the pool / projection / loss rows of the hot path.

TEST INFRASTRUCTURE ONLY (see oracle/retrieval.py).  numpy restatements, fp64 arithmetic;
pinned against golden vectors from the reference's own modules
(tests/golden/make_golden_model.py -> tests/golden/model_*.npz, tests/test_oracle_heads.py).
"""
from __future__ import annotations

import numpy as np

VIDEO_MAX_LEN = 64  # LINAS-engine/util/tag_data_provider.py:11


def collate_frame(frames_list):
    """LINAS-engine/util/tag_data_provider.py:91-109: pad/truncate to <=64, mean over ALL frames."""
    lengths = [min(VIDEO_MAX_LEN, len(f)) for f in frames_list]
    B, F, t_max = len(frames_list), frames_list[0].shape[1], max(lengths)
    videos = np.zeros((B, t_max, F))
    origin = np.zeros((B, F))
    mask = np.zeros((B, t_max))
    for i, f in enumerate(frames_list):
        e = lengths[i]
        videos[i, :e] = f[:e]
        origin[i] = np.mean(np.asarray(f, np.float64), 0)
        mask[i, :e] = 1.0
    return videos, origin, lengths, mask


def pool_mean_valid(x, lengths):
    """LINAS-engine/model.py:152-156."""
    return np.stack([np.mean(x[i, :lengths[i]], 0) for i in range(x.shape[0])])


def pool_masked_max(x, mask):
    """LINAS-engine/model.py:157-158: torch.max(x * mask, 1) -- masked steps contribute 0."""
    return np.max(x * mask[:, :, None], axis=1)


def pool_max(x):
    """LINAS-engine/model.py:166 (max_pool1d over the full padded length)."""
    return np.max(x, axis=1)


def pool_mean(x):
    """MultiFusion/src/combiner.py:140-143 time_process; MCT recognizer2d.py:76-83 TSN segment mean."""
    return np.mean(x, axis=1)


def tsn_feature_extraction(x, batches):
    """MCT/mmaction/models/recognizers/recognizer2d.py:76-83 (feature_extraction=True): the backbone maps
    x [batches * num_segs, C, H, W] -> AdaptiveAvgPool2d(1) (:78-79, a mean over H x W per plane) ->
    reshape (batches, num_segs, -1) (:81) -> mean over axis 1 (:83).  fp64.  MCT is not importable here
    (mmcv is absent): pinned against torch's own AdaptiveAvgPool2d + mean on the same maps
    (tests/test_oracle_heads.py), parity with a run of the reference itself unpinned."""
    x = np.asarray(x, np.float64)
    n, C = x.shape[:2]
    planes = x.reshape(n, C, -1).mean(axis=2)
    return planes.reshape(batches, n // batches, C).mean(axis=1)


def l2norm(x):
    """LINAS-engine/model.py:35-40 (no epsilon)."""
    return x / np.sqrt(np.sum(x * x, axis=1, keepdims=True))


def latent_mapping_eval(x, sd, layers, l2=True, bn_eps=1e-5):
    """LINAS-engine/model.py:97-116 (MFC eval) + :374-381 (Latent_mapping), from a state dict."""
    x = np.asarray(x, np.float64)
    n_fc = len(layers)
    f = x @ sd["mapping.fc1.weight"].T.astype(np.float64) + sd["mapping.fc1.bias"]
    for k in range(2, min(n_fc, 5)):
        w, b = sd[f"mapping.fc{k}.weight"], sd[f"mapping.fc{k}.bias"]
        f = f + np.maximum(f @ w.T.astype(np.float64) + b, 0.0)
    f = (f - sd["mapping.bn_1.running_mean"]) / np.sqrt(sd["mapping.bn_1.running_var"].astype(np.float64) + bn_eps) \
        * sd["mapping.bn_1.weight"] + sd["mapping.bn_1.bias"]
    return l2norm(f) if l2 else f


def triplet_loss(s, im, margin, max_violation, mean_style, direction):
    """LINAS-engine/loss.py:112-153 forward + the autograd backward.  Returns (loss, d_s, d_im).
    direction: 1 v2t (cost_s), 2 t2v (cost_im), 3 all."""
    s = np.asarray(s, np.float64)
    im = np.asarray(im, np.float64)
    S = im @ s.T
    B = S.shape[0]
    d = np.diag(S)
    eye = np.eye(B, dtype=bool)
    dS = np.zeros_like(S)
    loss = 0.0
    for bit, axis in ((1, 1), (2, 0)):
        if not direction & bit:
            continue
        raw = margin + S - (d[:, None] if axis == 1 else d[None, :])
        cost = np.where(eye, 0.0, np.maximum(raw, 0.0))
        act = (raw >= 0) & ~eye
        if max_violation:
            arg = np.argmax(cost, axis=axis)  # first index on ties, like torch.max
            val = np.take_along_axis(cost, np.expand_dims(arg, axis), axis).squeeze(axis)
            w = 1.0 / B if mean_style else 1.0
            loss += val.sum() * w
            sel = np.zeros_like(S, dtype=bool)
            if axis == 1:
                sel[np.arange(B), arg] = True
            else:
                sel[arg, np.arange(B)] = True
            g = (sel & act) * w
        else:
            w = 1.0 / (B * B) if mean_style else 1.0
            loss += cost.sum() * w
            g = act * w
        dS += g
        # -S_dd term of every active entry
        if axis == 1:
            dS[np.arange(B), np.arange(B)] -= g.sum(axis=1)
        else:
            dS[np.arange(B), np.arange(B)] -= g.sum(axis=0)
    return loss, dS.T @ im, dS @ s


def infonce(P, T, scale=100.0):
    """Row CE(scale * P T^T, arange) (MultiFusion/src/combiner_train.py:367-372) and col CE on the
    transpose; returns (row, col, dP_row, dT_row, dP_col, dT_col)."""
    P = np.asarray(P, np.float64)
    T = np.asarray(T, np.float64)
    L = scale * P @ T.T
    B = L.shape[0]

    def ce(Lm):
        m = Lm.max(axis=1, keepdims=True)
        lse = m[:, 0] + np.log(np.exp(Lm - m).sum(axis=1))
        loss = np.mean(lse - np.diag(Lm))
        G = (np.exp(Lm - lse[:, None]) - np.eye(B)) / B
        return loss, G

    row, Gr = ce(L)
    col, Gc = ce(L.T)
    Gc = Gc.T
    return row, col, scale * Gr @ T, scale * Gr.T @ P, scale * Gc @ T, scale * Gc.T @ P
