"""CPU: host-side logic of the drop-in API (argument validation with the reference's error
behaviour, config plumbing, the rank/ctr slot layout parse)."""
import json
import os

import pytest
import torch

from recommendsystem_amd.autoint import AutoIntConfig
from recommendsystem_amd.feature_config import SingleSlot, SlotLayout
from recommendsystem_amd.layers import InteractingLayer, MultiLayerDense, _act_code

REF_JSON = "/root/reference/rank/ctr/model_parameter.json"


def test_interacting_layer_rank_error_message():
    il = InteractingLayer(1, 16, 2)
    with pytest.raises(ValueError, match="The rank of input of InteractingLayer must be 3, but now is 2"):
        il(torch.zeros(2, 16))
    with pytest.raises(ValueError, match="must be 3, but now is 4"):
        il.build((1, 2, 3, 4))


def test_interacting_layer_head_split_and_tied_weights_errors():
    with pytest.raises(ValueError, match="evenly divisible"):
        InteractingLayer(1, 16, 3).build((2, 5, 16), device="cpu")
    with pytest.raises(ValueError, match="tied weights"):
        InteractingLayer(2, 8, 2).build((2, 5, 16), device="cpu")


def test_interacting_layer_defaults_match_reference():
    il = InteractingLayer()
    assert (il.layer_num, il.unit_num, il.head_num, il.use_dropout, il.dropout_rate, il.use_res) == \
        (1, 128, 1, False, 0.3, True)  # InteractingLayer.py:9-16


def test_layer_build_on_cpu_has_flat_grad_block():
    il = InteractingLayer(3, 16, 2)
    il.build((4, 26, 16), device="cpu")
    from recommendsystem_amd.params import grads_contiguous
    blk = grads_contiguous([il.kernel, il.bias, il.gamma, il.beta])
    assert blk is not None and blk.numel() == 16 * 64 + 64 + 32
    assert torch.all(il.gamma == 1) and torch.all(il.beta == 0) and torch.all(il.bias == 0)
    lim = (6.0 / (16 + 16)) ** 0.5  # glorot_uniform per Dense kernel
    assert float(il.kernel.detach().abs().max()) <= lim


def test_gpu_ops_refuse_cpu_tensors():
    from recommendsystem_amd._lib import RecsysKernelError
    il = InteractingLayer(1, 16, 2)
    il.build((2, 5, 16), device="cpu")
    with pytest.raises(RecsysKernelError):
        il(torch.zeros(2, 5, 16))


def test_activation_codes():
    assert _act_code("relu") == 1 and _act_code("sigmoid") == 2 and _act_code(None) == 0
    with pytest.raises(NotImplementedError):
        _act_code("tanh")
    m = MultiLayerDense([32, 16], "relu")
    assert [l.units for l in m.layers] == [32, 16]


def test_autoint_config_from_model_param():
    mc = {"model_param": {"interact": dict(layer_num=3, unit_num=16, head_num=2, use_dropout=False,
                                           dropout_rate=0.1, use_res=True),
                          "mlp": dict(hidden_units=[32, 16], activation="relu"),
                          "logits": dict(hidden_units=[1], activation="sigmoid")}}
    c = AutoIntConfig.from_model_config(mc, num_fields=26)
    assert (c.layer_num, c.unit_num, c.head_num, tuple(c.mlp_hidden), tuple(c.logits_hidden)) == \
        (3, 16, 2, (32, 16), (1,))


def test_single_slot_intervals():
    s = SingleSlot("1")
    s.update_intervals(8, True)
    s.update_intervals(16, False)  # bias feature: no structure interval
    s.update_intervals(4, True)
    assert s.intervals == [[0, 8], [24, 28]] and s.total_emb_size == 28


def _synthetic_config():
    return {"feature_slot": {
        "sparse_feature": {
            "a": {"slot_id": ["10"], "emb_size": 8},
            "b": {"slot_id": ["10"], "emb_size": 4, "bias": 1, "bias_type": "ppnet"},
            "c": {"slot_id": ["2"], "emb_size": 16},
            "d": {"slot_id": ["2"], "emb_size": 8, "bias": 1, "bias_type": "can"},
            "e": {"slot_id": ["7", "8"], "emb_size": 12},
        },
        "sequence_feature": {"s": {"slot_id": ["99"], "emb_size": 16}},
        "dense_feature": {"x": {"slot_id": "555"}},
    }}


def test_slot_layout_synthetic():
    L = SlotLayout.from_model_config(_synthetic_config())
    assert L.max_embed_size == 24
    assert L.structure_intervals() == [("10", 0, 8), ("2", 0, 16), ("7", 0, 12), ("99", 0, 16)]
    assert L.bias_intervals() == {"ppnet": [("10", 8, 12)], "can": [("2", 16, 24)]}
    assert L.sparse_slots == sorted(["10", "2", "7", "8", "99"])
    assert L.dense_slots == ["555"]
    cols = L.column_plan([("2", 0, 2), ("10", 8, 10)])
    pos = {s: i for i, s in enumerate(L.sparse_slots)}
    assert cols == [pos["2"] * 24, pos["2"] * 24 + 1, pos["10"] * 24 + 8, pos["10"] * 24 + 9]


def test_slot_layout_errors():
    cfg = _synthetic_config()
    cfg["feature_slot"]["sparse_feature"]["b"].pop("bias_type")
    with pytest.raises(Exception, match="bias_type could not be null"):
        SlotLayout.from_model_config(cfg)
    cfg = _synthetic_config()
    cfg["feature_slot"]["sequence_feature"]["s"]["slot_id"] = ["10"]
    with pytest.raises(Exception, match="has been defined more than once"):
        SlotLayout.from_model_config(cfg)


@pytest.mark.skipif(not os.path.exists(REF_JSON), reason="reference tree not mounted")
def test_slot_layout_on_reference_json():
    """Aggregates of the shipped rank/ctr/model_parameter.json quoted in SURVEY §8a H2."""
    L = SlotLayout.from_model_config(json.load(open(REF_JSON)))
    si = L.structure_intervals()
    assert L.max_embed_size == 96 and len(si) == 175 and sum(b - a for _, a, b in si) == 2500
    assert {k: sum(b - a for _, a, b in v) for k, v in L.bias_intervals().items()} == \
        {"ppnet": 272, "can": 176, "multiply_user": 48, "multiply_item": 48}


def test_rank_ctr_fixture_layout():
    """tests/golden/rank_ctr_feature_slot.json (the shipped model_parameter.json with anonymised
    feature names) yields the reference layout the GPU tests build the rank/ctr model on."""
    fx = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rank_ctr_feature_slot.json")
    L = SlotLayout.from_model_config(json.load(open(fx)))
    si = L.structure_intervals()
    assert L.max_embed_size == 96 and len(si) == 175 and sum(b - a for _, a, b in si) == 2500
    assert len(L.sparse_slots) == 176
    if os.path.exists(REF_JSON):
        R = SlotLayout.from_model_config(json.load(open(REF_JSON)))
        assert R.structure_intervals() == si and R.bias_intervals() == L.bias_intervals()
        assert R.sparse_slots == L.sparse_slots


def test_featureid_to_slot_data():
    from recommendsystem_amd.feature_config import FEATUREID_TO_SLOT, GATE_FEATURE_LIST
    assert len(FEATUREID_TO_SLOT) == 156 and FEATUREID_TO_SLOT["42285"] == "9517"
    assert FEATUREID_TO_SLOT["41189"] == FEATUREID_TO_SLOT["41187"] == "2602"  # shared slot
    assert len(GATE_FEATURE_LIST) == 16


def test_trainer_lr_groups_segments():
    """Trainer(lr_groups=...) splits the dense arena into contiguous learning-rate segments, each
    with its own step counter (config 5: the DSSM at rough_rank/model.py:209's lr 1e-4 beside the
    staytime towers' 5e-4)."""
    import torch
    from torch import nn
    from recommendsystem_amd.trainer import Trainer

    class Joint(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(3, 4)
            self.b = nn.Linear(4, 2)
            self.c = nn.Linear(2, 5)

    m = Joint()
    t = Trainer(m, 5e-4, lr_groups=[(m.b, 1e-4)])
    segs = [(o, n, lr) for o, n, lr, _ in t.segments]
    # layers led by a weight matrix start 16-float aligned (trainer.ARENA_ALIGN): a.weight 0..12,
    # a.bias 12..16, b.weight 16..24, b.bias 24..26, (gap) c.weight 32..42, c.bias 42..47
    assert segs == [(0, 16, 5e-4), (16, 10, 1e-4), (26, 21, 5e-4)]
    cnts = [c for *_, c in t.segments]
    assert cnts[0] is t.step_count and len({id(c) for c in cnts}) == 3
    assert [(o, n, lr) for o, n, lr, _ in Trainer(m, 5e-4).segments] == [(0, 47, 5e-4)]
    assert m.c.weight.data_ptr() % 64 == 0 or m.c.weight.data_ptr() - m.a.weight.data_ptr() == 128
