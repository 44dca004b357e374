"""CPU: the conv tuner's shape classes (VERDICT r4 Next #2b).  A key first seen at a new spatial size reuses
the winner of the nearest raced key of the same layer signature instead of timing every candidate again
(real COCO batches change H x W from step to step: /root/reference/train.py:197-214,377-378), and MIOpen's
candidates are out of the races by default (#2c)."""
import pytest

from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import ConvTuner


@pytest.fixture
def tuner(monkeypatch):
    for k in ("MXR_CONV_FORCE", "MXR_CONV_EXCLUDE", "MXR_CONV_NEAREST", "MXR_CONV_TABLE"):
        monkeypatch.delenv(k, raising=False)
    t = ConvTuner()
    monkeypatch.setattr(t, "_tuning_allowed", lambda: True)
    return t


def test_split_key_plain_and_pyramid():
    sig, px = ConvTuner.split_key("fwd|16|200|334|64|256|1|1|(0, 0, 0, 0)|1|1|eb")
    assert sig == "fwd|16|*|*|64|256|1|1|(0, 0, 0, 0)|1|1|eb" and px == 200 * 334
    sig, px = ConvTuner.split_key("pfwd|16|((100, 167), (50, 84))|256|256|1")
    assert sig == "pfwd|16|*|256|256|1" and px == 100 * 167 + 50 * 84
    assert ConvTuner.split_key("stem|16|x") is None


def test_split_key_projection_gemms():
    # the fused projection-block keys carry two grids (output and block input): both are spatial
    sig, px = ConvTuner.split_key("fwdp|16|100|167|128|256|512|2|200|334|eb")
    assert sig == "fwdp|16|*|*|128|256|512|2|*|*|eb" and px == 100 * 167
    sig2, _ = ConvTuner.split_key("fwdp|16|96|160|128|256|512|2|192|320|eb")
    assert sig2 == sig
    sig, px = ConvTuner.split_key("wgradp|16|50|84|256|512|1024|2|100|167|s")
    assert sig == "wgradp|16|*|*|256|512|1024|2|*|*|s" and px == 50 * 84
    assert ConvTuner.split_key("dgradp|16|50|84|1024") is None


def test_nearest_class_reused_without_racing(tuner):
    raced = "fwd|16|200|334|64|256|1|1|(0, 0, 0, 0)|1|1|eb"
    tuner.table[raced] = "hip14"
    tuner.timings[raced] = {"hip14": 0.29}
    new = "fwd|16|200|272|64|256|1|1|(0, 0, 0, 0)|1|1|eb"      # a 800 x 1088 batch's stage-2 key
    called = []
    cands = {n: (lambda n=n: called.append(n) or n) for n in ("hip11", "hip14", "c1x1_64")}
    assert not tuner.needs_tuning(new, cands)
    assert tuner.winner(new) == "hip14"
    assert tuner.run(new, cands) == "hip14" and called == ["hip14"]      # one call: no race
    assert tuner.table[new] == "hip14" and tuner.borrowed[new] == raced
    # another signature (cout differs) is not borrowed from
    other = "fwd|16|200|272|64|512|1|1|(0, 0, 0, 0)|1|1|eb"
    assert tuner.needs_tuning(other, cands) and tuner.winner(other) is None


def test_far_class_or_missing_candidate_races(tuner, monkeypatch):
    raced = "pfwd|16|((100, 167), (50, 84))|256|256|1"
    tuner.table[raced] = "hx32_0"
    far = "pfwd|16|((25, 42), (13, 21))|256|256|1"             # 15x fewer pixels: beyond the radius
    assert tuner.needs_tuning(far, ["hx32_0", "hx32_6"])
    near = "pfwd|16|((96, 160), (48, 80))|256|256|1"
    assert not tuner.needs_tuning(near, ["hx32_0", "hx32_6"])
    assert tuner.needs_tuning(near, ["hx32_6", "hx32_1"])       # the class winner is no candidate here
    monkeypatch.setenv("MXR_CONV_NEAREST", "0")                   # classes off: always race
    assert tuner.needs_tuning(near, ["hx32_0", "hx32_6"])


def test_borrowed_keys_are_not_sources(tuner):
    a = "dgrad|16|50|84|256|256|3|1|(1, 1, 1, 1)|m"
    tuner.table[a] = "hx32_6"
    b = "dgrad|16|48|84|256|256|3|1|(1, 1, 1, 1)|m"
    assert tuner.run(b, {"hx32_6": lambda: 1, "hx32_0": lambda: 0}) == 1
    del tuner.table[a]
    c = "dgrad|16|46|84|256|256|3|1|(1, 1, 1, 1)|m"
    assert tuner.winner(c) is None        # b was borrowed: no chain of borrowings


def test_miopen_out_of_races_by_default(tuner, monkeypatch):
    assert tuner._filter(["hip1", "miopen"]) == ["hip1"]
    assert tuner._filter(["miopen"]) == ["miopen"]                # the only implementation stays
    monkeypatch.setenv("MXR_CONV_EXCLUDE", "none")
    assert tuner._filter(["hip1", "miopen"]) == ["hip1", "miopen"]
    monkeypatch.setenv("MXR_CONV_FORCE", "miopen")                # a pinned family still runs
    monkeypatch.setenv("MXR_CONV_EXCLUDE", "miopen")
    assert tuner.run("fwd|1|2|2|64|64|1|1|(0, 0, 0, 0)|0|0", {"hip1": lambda: "h", "miopen": lambda: "m"}) == "m"


def test_winner_only_keys_adopt_and_do_not_rescan(tuner, monkeypatch):
    """A key that only goes through winner() (the fused weight + bias gradient path) adopts its class's
    winner at first sight; later calls are table hits, not scans of the whole table (the rescans cost ~25 ms
    per step on real COCO batches)."""
    raced = "pwgrad|16|((100, 167), (50, 84))|256|256|s"
    tuner.table[raced] = "hip24"
    scans = []
    real = tuner._nearest_scan
    monkeypatch.setattr(tuner, "_nearest_scan", lambda *a: scans.append(1) or real(*a))
    new = "pwgrad|16|((100, 134), (50, 67))|256|256|s"
    for _ in range(5):
        assert tuner.winner(new) == "hip24"
    assert len(scans) == 1 and tuner.table[new] == "hip24" and tuner.borrowed[new] == raced


def test_prefer_adopts_near_tie_only(tuner):
    """ConvTuner.prefer: a candidate whose form removes work outside the timed call (the fused focal epilogue,
    fp8-only tower outputs) replaces a raced winner within the margin -- re-timed medians when both have one --
    and never a clearly faster one; borrowed keys compare the source key's timings."""
    k = "pfwd|16|((100, 167), (50, 84))|256|720|0"
    assert not tuner.prefer(k, "hx32_0", 0.15)                    # untuned: nothing to prefer over
    tuner.table[k] = "hx32_4"
    tuner.timings[k] = {"hx32_4": 0.983, "hx32_0": 0.937, "hx32_4~": 0.930, "hx32_0~": 0.941, "hx32_6": 1.2}
    assert tuner.prefer(k, "hx32_0", 0.15)
    assert tuner.table[k] == "hx32_0" and tuner.preferred[k] == "hx32_4"
    assert tuner.prefer(k, "hx32_0", 0.0)                         # already the choice
    k2 = "pfwd|16|((100, 167), (50, 84))|256|256|1|f8"
    tuner.table[k2] = "f8_21"
    tuner.timings[k2] = {"f8_21": 0.20, "f8_20": 0.25}            # no re-timed pair: first-pass times
    assert not tuner.prefer(k2, "f8_20", 0.02) and tuner.table[k2] == "f8_21"
    assert tuner.prefer(k2, "f8_20", 0.06) and tuner.table[k2] == "f8_20"
    k3 = "pfwd|16|((96, 160), (48, 80))|256|720|0"                 # a shape class borrowing k's choice
    tuner.table[k] = "hx32_4"
    assert tuner.winner(k3) == "hx32_4" and tuner.borrowed[k3] == k
    assert tuner.prefer(k3, "hx32_0", 0.15) and tuner.table[k3] == "hx32_0"
    assert not tuner.prefer("pfwd|16|((7, 11),)|256|720|0", "hx32_0", 0.15)


def test_race_drops_borrowed_link_and_memo_follows_in_place_changes(tuner, monkeypatch):
    """(1) a key that borrowed its class's winner and is later raced (a caller whose candidates do not
    include the borrowed name) owns its timings from then on -- the borrowed link goes, so prefer() reads its own
    race and the key becomes a shape-class source; (2) a winner changed in place (prefer / sync) reaches the
    memoised borrowers."""
    raced = "fwd|16|200|334|64|256|1|1|(0, 0, 0, 0)|1|1|eb"
    tuner.table[raced] = "hip14"
    tuner.timings[raced] = {"hip14": 0.29, "hip11": 0.30}
    new = "fwd|16|200|272|64|256|1|1|(0, 0, 0, 0)|1|1|eb"
    assert tuner.winner(new) == "hip14" and tuner.borrowed[new] == raced
    monkeypatch.setattr("torch.cuda.synchronize", lambda *a: None)

    class _Ev:
        def __init__(self, **kw):
            pass

        def record(self):
            pass

        def synchronize(self):
            pass

        def elapsed_time(self, other):
            return 1.0
    monkeypatch.setattr("torch.cuda.Event", _Ev)
    assert tuner.run(new, {"c1p_1": lambda: "a", "c1p_2": lambda: "b"}) in ("a", "b")
    assert new not in tuner.borrowed and new in tuner.timings
    # in-place change of a source's winner: a memoised (not adopted) lookup follows it
    monkeypatch.setattr(tuner, "_tuning_allowed", lambda: False)
    other = "fwd|16|200|300|64|256|1|1|(0, 0, 0, 0)|1|1|eb"
    first = tuner.winner(other)
    src = tuner._nearest(other)[1]
    tuner.timings[src] = {first: 0.30, "hip99": 0.30}
    assert tuner.prefer(src, "hip99", 0.05)
    assert tuner.winner(other) == "hip99"
