"""CPU: no source file in the tree is git-ignored.  The round-3 queue harness
source was once matched by an ignore pattern meant for its built executable
and so never reached the history; this keeps every source the tests, the build
or the docs name under version control."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SOURCE_EXT = (".c", ".cc", ".cpp", ".h", ".hpp", ".hip", ".py", ".rs", ".sh", ".toml", ".md", ".json")
SKIP_DIRS = {".git", "__pycache__", ".pytest_cache", ".hypothesis", "gpurun_out", ".gpurun", "_build", "_ref", "lib"}


def test_no_source_is_ignored():
    if shutil.which("git") is None or not os.path.isdir(os.path.join(ROOT, ".git")):
        pytest.skip("not a git checkout")
    srcs = []
    for d, dirs, files in os.walk(ROOT):
        dirs[:] = [x for x in dirs if x not in SKIP_DIRS and not x.startswith("build")]
        srcs += [os.path.relpath(os.path.join(d, f), ROOT) for f in files if f.endswith(SOURCE_EXT)]
    r = subprocess.run(["git", "check-ignore", "--no-index", "--stdin"], cwd=ROOT, input="\n".join(srcs),
                       capture_output=True, text=True)
    ignored = [p for p in r.stdout.split("\n") if p and p not in ("PROGRESS.jsonl", "COPYCHECK.json")]
    assert not ignored, f"sources matched by .gitignore: {ignored}"
