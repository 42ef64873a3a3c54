"""REST handler mirror (keto_amd/handler.py): the reference's handler tests restated
(internal/check/handler_test.go:41-109, internal/expand/handler_test.go:30-108) plus the
batch-check endpoint.  URL parsing and expand run on CPU; check routes need the GPU."""
import json

import pytest

from keto_amd import _lib as L
from keto_amd import check, expand
from keto_amd import relationtuple as rt
from keto_amd.handler import BadRequest, Handler, relation_query_from_url, tuple_from_url
from keto_amd.snapshot import Snapshot


def q(**kw):
    return {k.replace("__", "."): [v] for k, v in kw.items()}


def test_url_query_parsing_matches_reference():
    # definitions.go:458-493
    with pytest.raises(BadRequest, match="support for \"subject\" was dropped"):
        relation_query_from_url({"subject": ["not#a valid userset rewrite"]})
    with pytest.raises(BadRequest, match="exactly one"):
        relation_query_from_url(q(subject_id="u", subject_set__namespace="n", subject_set__object="o",
                                  subject_set__relation="r"))
    with pytest.raises(BadRequest, match="incomplete subject"):
        relation_query_from_url(q(subject_set__namespace="n", subject_set__object="o"))
    assert relation_query_from_url(q(namespace="n", subject_id="u")) == ("n", "", "", rt.SubjectID("u"))
    assert relation_query_from_url(q(object="o", subject_set__namespace="n", subject_set__object="x",
                                     subject_set__relation="")) == ("", "o", "", rt.SubjectSet("n", "x", ""))
    with pytest.raises(BadRequest, match="Subject has to be specified"):
        tuple_from_url(q(namespace="n"))


@pytest.fixture
def expand_handler():
    ns = [("expand handler", 1)]
    tuples = [rt.InternalRelationTuple("expand handler", "root", "parent of", rt.SubjectID(f"child{i}"))
              for i in range(2)]
    return Handler(None, expand.Engine(Snapshot.from_tuples(ns, tuples)))


def test_expand_handler_matches_reference(expand_handler):
    h = expand_handler
    code, body = h.get_expand("max-depth=foo")  # handler_test.go:38-46
    assert code == 400 and "invalid syntax" in body["error"]["reason"]
    code, body = h.get_expand("max-depth=10&namespace=not+expand+handler")  # :48-59
    assert code == 404 and "Unknown namespace" in body["error"]["reason"]
    code, body = h.get_expand("namespace=expand+handler&object=root&relation=parent+of&max-depth=2")  # :61-107
    assert code == 200
    assert body == {"type": "union", "subject_set": {"namespace": "expand handler", "object": "root",
                                                     "relation": "parent of"},
                    "children": [{"type": "leaf", "subject_id": "child0"}, {"type": "leaf", "subject_id": "child1"}]}
    code, body = h.get_expand("namespace=expand+handler&object=nothing&relation=x&max-depth=2")
    assert code == 200 and body is None  # a nil tree is JSON null (cmd/expand/root_test.go)


@pytest.mark.gpu
def test_check_handler_matches_reference():
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    ns = [("check handler", 1)]
    snap = Snapshot.from_tuples(ns, [rt.InternalRelationTuple("check handler", "o", "r", rt.SubjectID("s"))])
    h = Handler(check.Engine(snap), expand.Engine(snap))
    assert h.get_check("subject=not%23a+valid+userset+rewrite")[0] == 400  # handler_test.go:54-61
    code, body = h.get_check("")  # :63-71
    assert code == 400 and "Subject has to be specified" in body["error"]["reason"]
    assert h.get_check("namespace=not+check+handler&subject_id=foo") == (403, {"allowed": False})  # :73-81
    assert h.get_check("namespace=check+handler&object=o&relation=r&subject_id=s") == (200, {"allowed": True})
    assert h.get_check("namespace=check+handler&subject_id=foo") == (403, {"allowed": False})  # :100-108
    # wildcard object/relation scan the whole namespace (R5)
    assert h.get_check("namespace=check+handler&subject_id=s") == (200, {"allowed": True})
    assert h.post_check(b'{"namespace":"check handler","object":"o","relation":"r","subject_id":"s"}')[0] == 200
    assert h.post_check(b"{not json")[0] == 400


@pytest.mark.gpu
def test_batch_endpoint_matches_single_checks():
    from tests import randgraph
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows = randgraph.make_graph(81, n_rows=800, n_obj=30, n_users=40, poison=True)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    h = Handler(check.Engine(snap), expand.Engine(snap))
    reqs = randgraph.make_requests(81, namespaces, rows, n=500)
    items = [{"namespace": ns, "object": o, "relation": r, **s} for ns, o, r, s in reqs]
    items.insert(3, {"namespace": "n0", "object": "o1", "relation": "r0"})  # no subject: inline 400
    code, body = h.post_check_batch(json.dumps({"tuples": items}).encode())
    assert code == 200
    res = body["results"]
    assert res[3]["error"]["code"] == 400
    want = randgraph.oracle_store(namespaces, rows).check_batch(reqs)
    got = [r["allowed"] for i, r in enumerate(res) if i != 3]
    assert got == [bool(x) for x in want]
    for i in (0, 1, 2, 10, 200):  # the same answers one request at a time
        it = items[i]
        assert h.post_check(json.dumps(it).encode())[1]["allowed"] == res[i]["allowed"]
