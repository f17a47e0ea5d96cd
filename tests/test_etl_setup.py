import json
import os
import random

from dnn_page_vectors_amd.config import Configuration
from dnn_page_vectors_amd.data import etl
from dnn_page_vectors_amd.experiment import SetupExperiment
from dnn_page_vectors_amd.io.vocab import load_vocab


def test_collect_assessment():
    recs = [{"query": "q1", "results": [{"url": "a", "assessment": "Vital"}, {"url": "b", "assessment": "Not found"},
                                        {"url": "c", "assessment": "Foreign language"},
                                        {"url": "d", "assessment": "Useful"}]},
            {"query": "q2", "results": [{"url": "e", "assessment": "Relevant"}, {"url": "f", "assessment": "Off-topic / Useless"},
                                        {"url": "g", "assessment": "Off-topic / Useless"},
                                        {"url": "h", "assessment": "Off-topic / Useless"}]}]
    rows = list(etl.collect_assessment(recs, random.Random(0)))
    q1 = [r for r in rows if r["q"] == "q1"]
    assert {r["corr_url"] for r in q1} == {"a", "d"} and len(q1) == 6  # 3 rows per positive (bug fixed)
    for r in q1:
        assert "b" in r["incorr_url"] and "a" not in r["incorr_url"] and "d" not in r["incorr_url"] and len(r["incorr_url"]) == 3
    q2 = [r for r in rows if r["q"] == "q2"]
    assert len(q2) == 1 and q2[0]["incorr_url"] == ["f", "g", "h"]


def test_type1_type3_and_join():
    rec = {"q": "hotel", "doc_corr": {"u1": "clarion hotel"}, "doc_incorr": {"u2": "bank", "u3": "x", "u4": "y"}}
    assert list(etl.collect_type1([rec])) == [{"q": "hotel", "corr_url": "u1", "incorr_url": ["u2", "u3", "u4"]}]
    assert list(etl.collect_type1([rec], as_text=True))[0]["doc_incorr"] == ["bank", "x", "y"]
    rows = list(etl.collect_type3(["q\tu1 u2\n", "r\tu3 u4 u5 u6 u7\n", "bad line\n"], random.Random(1)))
    assert len(rows) == 2 * 3 + 5 * 3
    for r in rows:
        assert r["corr_url"] not in r["incorr_url"]
    pages = etl.read_page_info_tsv([json.dumps(u) + "\t" + json.dumps({"title": f"T{u}", "desc": "d", "url_words": u,
                                                                       "top_n_q": ["x"]}) + "\n"
                                    for u in ["u1", "u2", "u3", "u4"]])
    joined = list(etl.join_pages([{"q": "hotel", "corr_url": "u1", "incorr_url": ["u2", "u3", "u4"]}], pages))
    assert joined == [{"q": "hotel", "doc_corr": "Tu1 d u1", "doc_incorr": ["Tu2 d u2", "Tu3 d u3", "Tu4 d u4"]}]


def test_setup_experiment_split_and_vocab(tmp_path):
    cfg = Configuration(experiment_root_directory=str(tmp_path), feature_level="word")
    src = tmp_path / "in.jsonl"
    rows = [{"q": f"q {i}", "doc_corr": f"doc {i}", "doc_incorr": ["a", "b", "c"]} for i in range(50)]
    src.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    exp = SetupExperiment(cfg)
    exp.create_workspace()
    for d in (cfg.data_dir, cfg.trained_model_dir, cfg.pickle_files_dir, cfg.vectors_directory):
        assert os.path.isdir(d)
    exp.import_dataset(str(src))
    nt, nv = exp.split_dataset_file()
    assert (nt, nv) == (41, 9)  # int(50*0.8)+1 train rows
    exp2 = SetupExperiment(Configuration(experiment_root_directory=str(tmp_path / "b"), feature_level="word"))
    exp2.create_workspace()
    exp2.import_dataset(str(src))
    exp2.split_dataset_file()
    assert open(cfg.model_training_data).read() == open(exp2.conf.model_training_data).read()  # seeded
    v = exp.build_vocabulary()
    assert load_vocab(cfg).itos == v.itos and "doc" in v.stoi
