"""H2 host logic: the rank/ctr BaseModel front-end layout (rank/ctr/base_model.py:14-159).

The reference parses model_parameter.json['feature_slot'] into per-slot embedding intervals:
every sparse feature appends `emb_size` columns to its slot's row (SingleSlot.update_intervals,
base_model.py:14-27); non-bias features become "structure" fields (emb_structure_input), bias
features (with a bias_type) become named bias groups (emb_bias_input); sequence features get a
slot of their own; every slot's table row is max_embed_size wide (the embedding_column dimension,
base_model.py:82-86, 209-210); feature ids listed in featureid_to_slot share another slot's table
(base_model.py:89-102).

``SlotLayout`` restates that parse (same iteration orders, same errors) and turns it into the
device-side plan: one table per slot of width max_embed_size and the column intervals that the
front end gathers into the concatenated activation (rs_gather_columns, csrc/front_end.hip).
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class SingleSlot:
    """rank/ctr/base_model.py:14-27."""
    slot_id: str
    intervals: list = field(default_factory=list)
    last_start: int = -1
    last_end: int = -1
    total_emb_size: int = 0

    def update_intervals(self, emb_size: int, is_single: bool) -> None:
        self.last_start = self.last_end + 1
        self.last_end = self.last_start + emb_size - 1
        if is_single:
            self.intervals.append([self.last_start, self.last_end + 1])
        self.total_emb_size += emb_size


@dataclass
class SlotLayout:
    slots: dict                    # slot_id -> SingleSlot (insertion order = JSON order)
    bias: dict                     # slot_id -> {bias_type: [start, end)}
    sparse_slots: list             # sorted feature ids that get an input (base_model.py:75-77)
    dense_slots: list              # dense feature slot ids (base_model.py:79-81)
    max_embed_size: int            # base_model.py:82-86

    @staticmethod
    def from_model_config(model_config: dict) -> "SlotLayout":
        fs = model_config["feature_slot"]
        sparse_features = fs["sparse_feature"]
        slots: dict = {}
        bias: dict = {}
        sparse_list: list = []
        for k in sparse_features.keys():                                   # :38
            feat = sparse_features[k]
            slot = feat["slot_id"][0]
            is_single = "bias" not in feat
            if slot in slots:
                slots[slot].update_intervals(feat["emb_size"], is_single)
            else:
                ss = SingleSlot(slot)
                ss.update_intervals(feat["emb_size"], is_single)
                slots[slot] = ss
            if "bias" in feat:                                              # :45-52
                if "bias_type" not in feat:
                    raise Exception("bias_type could not be null")
                bt = feat["bias_type"]
                bias.setdefault(slot, {})[bt] = [slots[slot].last_start, slots[slot].last_end + 1]
            for s in set(feat["slot_id"]):
                sparse_list.append(s)
        seq_list: list = []
        for k in fs["sequence_feature"].keys():                            # :58-68
            feat = fs["sequence_feature"][k]
            slot = feat["slot_id"][0]
            if slot not in slots:
                ss = SingleSlot(slot)
                ss.update_intervals(feat["emb_size"], True)
                slots[slot] = ss
            else:
                raise Exception("sequence feature " + slot + "has been defined more than once")
            for s in set(feat["slot_id"]):
                seq_list.append(s)
        sparse_slots = sorted(set(sparse_list + seq_list))                  # :70-73
        dense_slots = [fs["dense_feature"][k]["slot_id"] for k in fs["dense_feature"].keys()]
        max_embed = max((s.total_emb_size for s in slots.values()), default=0)
        return SlotLayout(slots, bias, sparse_slots, dense_slots, max_embed)

    # ---- the activations the reference builds (base_model.py:134-154) ----
    def structure_intervals(self) -> list:
        """[(slot, start, end)] in emb_structure_input order (slot insertion order, then
        interval order)."""
        return [(slot, a, b) for slot, ss in self.slots.items() for a, b in ss.intervals]

    def bias_intervals(self) -> dict:
        """{bias_type: [(slot, start, end)]} in emb_bias_input order (sorted slots, then the
        slot's bias types in insertion order)."""
        out: dict = {}
        for slot in sorted(self.bias.keys()):
            for bt, (a, b) in self.bias[slot].items():
                out.setdefault(bt, []).append((slot, a, b))
        return out

    def gate_intervals(self, gate_feature_list) -> list:
        return [(slot, a, b) for slot, a, b in self.structure_intervals() if slot in gate_feature_list]

    def column_plan(self, intervals, slot_order=None) -> list:
        """Source column (into the [B, n_slots * max_embed_size] slot-major lookup output) of every
        concatenated output column, for rs_gather_columns."""
        order = slot_order or self.sparse_slots
        pos = {s: i for i, s in enumerate(order)}
        cols = []
        for slot, a, b in intervals:
            base = pos[slot] * self.max_embed_size
            cols.extend(range(base + a, base + b))
        return cols
