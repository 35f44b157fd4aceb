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
front end gathers into the concatenated activation (rs_gather_columns, csrc/front_end.hip;
consumed by rank_models.RankCtrFrontEnd).
"""
from __future__ import annotations

from dataclasses import dataclass, field


# featureid_to_slot (rank/ctr/base_model.py:89): feature ids whose FeatureSlot -- hence embedding
# table -- is another slot's (data of the shipped model; sorted by feature id here)
FEATUREID_TO_SLOT: dict = {
    "40545": "7777", "40546": "7778", "40547": "7779", "40549": "7781", "40550": "7782", "40551": "7783",
    "40850": "8082", "40880": "8112", "40882": "8114", "40883": "8115", "40884": "8116", "40885": "8117",
    "40886": "8118", "40887": "8119", "40888": "8120", "40893": "8125", "40894": "8126", "40904": "8136",
    "40905": "8137", "40907": "8139", "40908": "8140", "40941": "8173", "40942": "8174", "40943": "8175",
    "40944": "8176", "40945": "8177", "40946": "8178", "40947": "8179", "40948": "8180", "40949": "8181",
    "40950": "8182", "40951": "8183", "40952": "8184", "40953": "8185", "40954": "8186", "40955": "8187",
    "41119": "8351", "41120": "8352", "41121": "8353", "41122": "8354", "41123": "8355", "41129": "8361",
    "41130": "8362", "41131": "8363", "41132": "8364", "41133": "8365", "41171": "3306", "41187": "2602",
    "41188": "2602", "41189": "2602", "41196": "3306", "41202": "3306", "41222": "8454", "41223": "8455",
    "41225": "8457", "41229": "3305", "41230": "3305", "41231": "8463", "41232": "3305", "41233": "8465",
    "41234": "8466", "41235": "8467", "41236": "8468", "41237": "8469", "41238": "8470", "41239": "8471",
    "41240": "8472", "41241": "8473", "41242": "8474", "41243": "8475", "41244": "8476", "41245": "8477",
    "41246": "8478", "41247": "8479", "41248": "8480", "41249": "8481", "41250": "8482", "41251": "8483",
    "41252": "8484", "41253": "8485", "41262": "8494", "41263": "8495", "41264": "8496", "41265": "8497",
    "41266": "8498", "41267": "8499", "41268": "8500", "41269": "8501", "41270": "8502", "41271": "8503",
    "41283": "8515", "41296": "8528", "41300": "8532", "41303": "8535", "41313": "8545", "41331": "8563",
    "41339": "8571", "41341": "8573", "41674": "3303", "41675": "3303", "41676": "3303", "41831": "9063",
    "41832": "9064", "41833": "9065", "41834": "9066", "41835": "9067", "41836": "9068", "41837": "9069",
    "41838": "9070", "41839": "9071", "41840": "9072", "41841": "9073", "41842": "9074", "41854": "9086",
    "41855": "9087", "41856": "9088", "41857": "9089", "41858": "9090", "41859": "9091", "41860": "9092",
    "41861": "9093", "42283": "9515", "42284": "9516", "42285": "9517", "42286": "9518", "42287": "9519",
    "42288": "9520", "42289": "9521", "42290": "9522", "42291": "9523", "42292": "9524", "42293": "9525",
    "42294": "9526", "42295": "9527", "42296": "9528", "42297": "9529", "42298": "9530", "42299": "9531",
    "42300": "9532", "42301": "9533", "42302": "9534", "42303": "9535", "42304": "9536", "42305": "9537",
    "42306": "9538", "42307": "9539", "42308": "9540", "42309": "9541", "42310": "9542", "42311": "9543",
    "42312": "9544", "42313": "9545", "42314": "9546", "42315": "9547", "42316": "9548", "42317": "9549",
}

# gate_feature_list (rank/ctr/base_model.py:122): structure fields that also feed the ppnet gate
# input of the MMoE experts (duplicates kept as the reference lists them; membership is what
# counts)
GATE_FEATURE_LIST: tuple = ("1568", "1570", "1578", "1591", "1593", "1614", "1736", "1737", "2039", "2599", "3051", "3303", "3389", "1576", "1577", "1578")


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

# staytime Config.SLOTS / SEQ_SLOTS (staytime/config.py:4-16): the VarLen int64 slots of
# parse_input_func (parse.py:22-23) and the behaviour sequences (data.dataset_reader's default)
STAYTIME_SLOTS = (
    '1568', '1570', '1571', '1574', '1575', '1576', '1577', '1578', '1579', '1581', '1582',
    '1583', '1585', '1587', '1589', '1591', '1592', '1593', '1594', '1595', '1599', '1601',
    '1611', '1612', '1614', '1616', '1623', '1636', '1736', '1737', '1738', '1739', '1740',
    '1741', '1743', '1744', '1749', '2039', '2040', '2041', '2042', '2043', '2044', '2050',
    '2051', '2052', '2123', '2125', '2127', '2128', '2130', '2131', '2135', '2139', '2142',
    '2144', '2147', '2149', '2151', '2152', '2154', '2156', '2544', '2597', '3051', '3365',
    '3369', '3376', '3370', '1745', '2045', '1632', '1735', '2153', '2047', '2244', '2046',
    '2150', '2247', '1625', '1624', '2148', '2159', '2146', '2242', '2260', '2155', '2259',
    '2615', '4500', '4386',
)
STAYTIME_SEQ_SLOTS = ('2125', '2128', '2130')
