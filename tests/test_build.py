"""Build hygiene: rebuilds are decided by content-hash stamps, not mtimes."""
import os
import time

import pytest

from mlapi_amd import _build


def test_stamp_is_content_not_mtime(tmp_path):
    out = tmp_path / "obj.o"
    out.write_bytes(b"object")
    dig = _build._digest(b"source bytes", "headers", "hipcc", ["-O3"])
    _build._write_stamp(out, dig)
    assert _build._stamp_ok(out, dig)
    # a fresh mtime on the same content does not trigger a rebuild ...
    later = time.time() + 3600
    os.utime(out, (later, later))
    assert _build._stamp_ok(out, dig)
    # ... and an object newer than its source is NOT reused when the source bytes changed
    assert not _build._stamp_ok(out, _build._digest(b"source bytes!", "headers", "hipcc", ["-O3"]))
    # flags and headers are part of the stamp too
    assert not _build._stamp_ok(out, _build._digest(b"source bytes", "headers", "hipcc", ["-O2"]))
    assert not _build._stamp_ok(out, _build._digest(b"source bytes", "headers2", "hipcc", ["-O3"]))


def test_missing_object_or_stamp_rebuilds(tmp_path):
    out = tmp_path / "obj.o"
    dig = _build._digest(b"x")
    assert not _build._stamp_ok(out, dig)  # no object
    out.write_bytes(b"o")
    assert not _build._stamp_ok(out, dig)  # object without a stamp (e.g. a prebuilt copy)


def test_in_tree_extension_matches_sources():
    """The extension that build() left in the tree was built from exactly these sources."""
    if not _build.ext_path().exists():
        pytest.skip("extension not built")
    assert _build.stamp_matches()
