"""(ix) MultiFusion ranking fixture: restated MultiFusion/src/validate.py:44-138 on the shipped val split.

MultiFusion/src/validate.py is NOT importable here (it imports OpenAI `clip`, `decord`, `h5py`,
`comet_ml`, none installed), so the expected recalls come from a literal torch restatement of its
lines 44-105 (time_process in chunks of 128, F.normalize, 1 - pred @ index.T, torch.argsort,
reference removal, top-50 labels, validate.py:135-138) over the first 256 triplets of
dataset/modified_dataset/vdo_modified_text_val_clip_remaped.txt and a 2,048-video sub-gallery.
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_multifusion.py /root/reference
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import synth  # noqa: E402


def literal_recalls(pred, index_features, index_names, reference_names, target_names):
    b = 128
    tmp = []
    for bt in range(int(len(index_features) / b) + 1):
        tmp.append(index_features[bt * b:(bt + 1) * b].mean(dim=1))  # combiner.time_process
    index = F.normalize(torch.cat(tmp, 0), dim=-1).float()
    b = 32
    labels = []
    names_t = torch.tensor(index_names)
    for bt in range(int(len(pred) / b) + 1):
        p = pred[bt * b:(bt + 1) * b]
        if len(p) == 0:
            continue
        dist = 1 - p @ index.T
        order = torch.argsort(dist.cpu(), dim=-1)
        sn = names_t[order]
        refs = torch.tensor(reference_names[bt * b:(bt + 1) * b])
        mask = sn != refs.unsqueeze(1).repeat(1, len(index_names))
        sn = sn[mask].reshape(sn.shape[0], sn.shape[1] - 1)
        tg = torch.tensor(target_names[bt * b:(bt + 1) * b])
        labels.append(sn[:, :50] == tg.unsqueeze(1).repeat(1, 50))
    labels = torch.cat(labels)
    return [(torch.sum(labels[:, :k]) / len(labels)).item() * 100 for k in (1, 5, 10, 50)]


def main(ref_root):
    tsv = os.path.join(ref_root, "MultiFusion", "dataset", "modified_dataset", "vdo_modified_text_val_clip_remaped.txt")
    rows = [l.rstrip("\n").split("\t") for l in open(tsv).readlines()[:256]]
    names, feats, pred, refs, tgts = synth.multifusion_ranking_case(rows)
    rec = literal_recalls(torch.from_numpy(pred), torch.from_numpy(feats), names.tolist(), refs, tgts)
    out = dict(names=names, refs=np.array(refs), tgts=np.array(tgts), recalls=np.array(rec),
               triplet_idx=np.array([int(r[0]) for r in rows]))
    path = os.path.join(HERE, "multifusion_rank.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, rec)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
