"""The runtime-knob registry (utils/knobs.py) covers every PAGEVEC_* environment variable the
package reads, so a bench record's `runtime_knobs` can say which ones a run changed."""
import glob
import os
import re

from dnn_page_vectors_amd.utils import knobs

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_READ = re.compile(r'environ(?:\.get)?\(\s*"(PAGEVEC_[A-Z0-9_]+)"|environ\[\s*"(PAGEVEC_[A-Z0-9_]+)"\]')


def test_every_env_knob_is_registered():
    names = set()
    files = glob.glob(os.path.join(REPO, "dnn_page_vectors_amd", "**", "*.py"), recursive=True)
    for f in files + [os.path.join(REPO, "bench.py")]:
        with open(f) as fh:
            for m in _READ.finditer(fh.read()):
                names.add(m.group(1) or m.group(2))
    for f in glob.glob(os.path.join(REPO, "dnn_page_vectors_amd", "csrc", "**", "*.hip"), recursive=True):
        with open(f) as fh:  # the kernels' own getenv() knobs
            names.update(re.findall(r'getenv\("(PAGEVEC_[A-Z0-9_]+)"\)', fh.read()))
    assert names, "no knob reads found (pattern out of date?)"
    missing = sorted(names - set(knobs.KNOBS))
    assert not missing, f"register these in utils/knobs.py: {missing}"
    for name, (kind, default, what) in knobs.KNOBS.items():
        assert kind in ("ab", "runtime", "hip") and isinstance(default, str) and what, name


def test_in_effect_and_non_default(monkeypatch):
    monkeypatch.setenv("PAGEVEC_CONV_SHORT", "0")
    monkeypatch.setenv("PAGEVEC_SOMETHING_UNREGISTERED", "x")
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    eff = knobs.in_effect()
    assert eff["PAGEVEC_CONV_SHORT"] == "0" and eff["PAGEVEC_SOMETHING_UNREGISTERED"] == "x"
    assert eff["GPU_MAX_HW_QUEUES"] == "4 (unset)"
    assert knobs.non_default().get("PAGEVEC_CONV_SHORT") == "0"
