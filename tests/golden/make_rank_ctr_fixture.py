"""Writes tests/golden/rank_ctr_feature_slot.json: the `feature_slot` section of the shipped
rank/ctr/model_parameter.json (/root/reference/rank/ctr/model_parameter.json) with the feature
NAMES replaced by f000, f001, ... (names do not enter the layout; order, slot ids, emb_size, bias
and bias_type do).  Data for the GPU tests of the rank/ctr model (the reference tree is not on
the GPU box).  Run from the repo root: python tests/golden/make_rank_ctr_fixture.py"""
import json
import os

SRC = "/root/reference/rank/ctr/model_parameter.json"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rank_ctr_feature_slot.json")

fs = json.load(open(SRC))["feature_slot"]
out = {}
for sec, feats in fs.items():
    out[sec] = {f"f{i:03d}": v for i, v in enumerate(feats.values())}
with open(OUT, "w") as f:
    json.dump({"feature_slot": out}, f, indent=0, sort_keys=False)
print("wrote", OUT)
