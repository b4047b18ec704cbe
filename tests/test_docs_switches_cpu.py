"""Every environment variable the package, the extension and bench.py read is in the runtime-switch table of
docs/ARCHITECTURE.md section 9 (the table is the user-facing list of toggles; an undocumented switch is a gap)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-llm-training-benchmark-framework_amd")
READ = re.compile(r"""(?:environ\.get|environ\[|getenv|environ\.setdefault)\(?\s*["'](DLTB_[A-Z0-9_]+)["']""")


def _sources():
    for base in (PKG, os.path.join(ROOT, "csrc")):
        for d, _, fs in os.walk(base):
            for f in fs:
                if f.endswith((".py", ".hip", ".cpp", ".h")):
                    yield os.path.join(d, f)
    yield os.path.join(ROOT, "bench.py")


def test_every_env_switch_is_documented():
    names = set()
    for p in _sources():
        names |= set(READ.findall(open(p, encoding="utf-8", errors="replace").read()))
    assert len(names) >= 20, names                       # the scan itself works
    doc = open(os.path.join(ROOT, "docs", "ARCHITECTURE.md"), encoding="utf-8").read()
    table = doc[doc.index("## 9. Runtime switches"):doc.index("## 10.")]
    missing = sorted(n for n in names if f"`{n}`" not in table and n not in table)
    assert not missing, f"undocumented runtime switches: {missing}"
