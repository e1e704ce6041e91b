"""Every ARENA_* environment switch the code reads is documented (docs/userguide.md or
docs/architecture.md): a knob nobody can find is dead weight (round-5 review, weak item 6)."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
_READ = re.compile(r'(?:environ(?:\.get)?\(\s*|environ\[\s*|getenv\(\s*)["\'](ARENA_[A-Z0-9_]+)["\']')


def _sources():
    yield from ROOT.glob("arena_amd/**/*.py")
    yield ROOT / "bench.py"
    yield from ROOT.glob("csrc/**/*.cpp")
    yield from ROOT.glob("csrc/**/*.hip")


def test_every_env_knob_is_documented():
    read = {}
    for p in _sources():
        for m in _READ.finditer(p.read_text(errors="ignore")):
            read.setdefault(m.group(1), p.relative_to(ROOT).as_posix())
    assert len(read) > 20   # the scan itself still finds the knobs
    docs = "".join((ROOT / "docs" / f).read_text() for f in ("userguide.md", "architecture.md"))
    missing = {k: v for k, v in read.items() if k not in docs}
    assert not missing, f"undocumented env knobs: {missing}"
