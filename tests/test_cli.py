"""`keto check` mirror with a batch mode (keto_amd/cli.py).
CPU: the tuple-file parser against the reference's parseFile rules (cmd/relationtuple/
parse.go:47-87) and the argument checks; GPU: single and batch checks against the oracle."""
import io
import json

import pytest

from keto_amd import _lib as L
from keto_amd import cli
from keto_amd import relationtuple as rt
from tests import randgraph

CAT_VIDEOS = """// contrib/cat-videos-example/relation-tuples (config #1)
videos:/cats/1.mp4#owner@videos:/cats#owner
videos:/cats/1.mp4#view@(videos:/cats/1.mp4#owner)
videos:/cats/1.mp4#view@*

videos:/cats/2.mp4#owner@videos:/cats#owner
videos:/cats/2.mp4#view@(videos:/cats/2.mp4#owner)
videos:/cats#owner@cat lady
videos:/cats#view@(videos:/cats#owner)
"""


def test_parse_file_follows_parse_go(tmp_path):
    p = tmp_path / "t.txt"
    p.write_text(CAT_VIDEOS)
    got = cli.parse_file(str(p))
    assert len(got) == 7
    assert got[1] == rt.InternalRelationTuple("videos", "/cats/1.mp4", "view", rt.SubjectSet("videos", "/cats/1.mp4",
                                                                                              "owner"))
    assert got[2].subject == rt.SubjectID("*") and got[5].subject == rt.SubjectID("cat lady")
    bad = tmp_path / "bad.txt"
    bad.write_text("a:b#c@d\n\n  no colon here  \n")
    err = io.StringIO()
    with pytest.raises(cli.CliError):
        cli.parse_file(str(bad), stderr=err)
    assert err.getvalue().startswith(f"Could not decode {bad}:3\n  no colon here\n")
    assert cli.parse_file("-", stdin=io.StringIO("n:o#r@s\n")) == [rt.InternalRelationTuple("n", "o", "r",
                                                                                            rt.SubjectID("s"))]


def test_arguments(tmp_path):
    err = io.StringIO()
    assert cli.main(["check", "a", "b", "c"], stderr=err) == 1 and "accepts 4 arg(s)" in err.getvalue()
    assert cli.main(["check", "a", "b", "c", "d", "--batch", "x"], stderr=io.StringIO()) == 1
    assert cli.main(["check", "a", "b", "c", "d"], stderr=io.StringIO()) == 1  # no network given
    err = io.StringIO()
    assert cli.main(["check", "--batch", str(tmp_path / "missing"), "--tuples", "t"], stderr=err) == 1
    assert "Could not open file" in err.getvalue()


@pytest.mark.gpu
def test_cli_single_and_batch_match_oracle(tmp_path):
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    t = tmp_path / "net.txt"
    t.write_text(CAT_VIDEOS)
    out = io.StringIO()
    base = ["--tuples", str(t), "--namespaces", "videos:0"]
    assert cli.main(["check", "cat lady", "view", "videos", "/cats/2.mp4"] + base, stdout=out) == 0
    assert out.getvalue() == "Allowed\n"  # SURVEY 8(c) config #1 expectations
    out = io.StringIO()
    cli.main(["check", "*", "view", "videos", "/cats/2.mp4", "--format", "json"] + base, stdout=out)
    assert json.loads(out.getvalue()) == {"allowed": False}
    # batch over a random network (no wildcard roots in the tuple format), every line
    namespaces, rows = randgraph.make_graph(91, n_rows=700, n_obj=30, n_users=40, wildcard=False)
    id2name = {i: n for n, i in namespaces}
    lines = [f"{id2name[ns]}:{o}#{r}@" + (sid if sid is not None else f"({id2name[sns]}:{so}#{sr})")
             for ns, o, r, sid, sns, so, sr in rows]
    t.write_text("\n".join(lines))
    reqs = randgraph.make_requests(91, namespaces, rows, n=400, wildcard=False)
    reqs = [q for q in reqs if q[0] in id2name.values()]
    q = tmp_path / "q.txt"
    q.write_text("\n".join(rt.InternalRelationTuple(ns, o, r, rt.subject_from_dict(s)).String() for ns, o, r, s in reqs))
    out = io.StringIO()
    spec = ",".join(f"{n}:{i}" for n, i in namespaces)
    assert cli.main(["check", "--batch", str(q), "--tuples", str(t), "--namespaces", spec], stdout=out) == 0
    want = randgraph.oracle_store(namespaces, rows).check_batch(reqs)
    assert out.getvalue().split("\n")[:-1] == ["Allowed" if x else "Denied" for x in want]
