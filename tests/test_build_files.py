"""meson.build (the reference's build system, /root/reference/meson.build:1-30) must list the same
sources the Makefile's wildcards compile: meson is absent from this image, so this is the check
that keeps the mirror from going stale."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _meson_paths():
    text = (ROOT / "meson.build").read_text()
    body = "\n".join(line.split("#", 1)[0] for line in text.splitlines())
    return set(re.findall(r"'([\w./]+\.(?:hip|hpp|cpp|c|h))'", body))


def _tree(pattern):
    return {p.relative_to(ROOT).as_posix() for p in ROOT.glob(pattern)}


def test_meson_lists_every_source():
    listed = _meson_paths()
    expected = (_tree("newsched_amd/csrc/*.hip") | _tree("newsched_amd/csrc/*.hpp")
                | _tree("newsched_amd/runtime/lib/*.cpp") | _tree("newsched_amd/schedulers/lib/*.cpp")
                | _tree("newsched_amd/blocklib/lib/*.cpp") | _tree("newsched_amd/capi/*.cpp")
                | _tree("tests/cpp/*.cpp") | _tree("tests/cpp/*.c") | _tree("tests/cpp/*.hip") | {"oracle/nsh_oracle.c", "include/nsh_hip.h",
                                               "include/nsr_flowgraph.h"})
    # tools are listed by stem ('tools' / name + '.cpp')
    tools = {f"tools/{n}.cpp" for n in re.findall(r"'(\w+)'", re.search(
        r"foreach name : \[([^\]]*)\]", (ROOT / "meson.build").read_text()).group(1))}
    assert tools == _tree("tools/*.cpp")
    assert expected - listed == set(), "meson.build is missing sources"
    assert listed - expected == set(), "meson.build names files that do not exist"


def test_meson_options_declared():
    opts = (ROOT / "meson_options.txt").read_text()
    used = set(re.findall(r"get_option\('(\w+)'\)", (ROOT / "meson.build").read_text()))
    builtin = {"libdir"}
    for name in used - builtin:
        assert f"option('{name}'" in opts, name
