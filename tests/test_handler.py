"""REST handler mirror (keto_amd/handler.py): the reference's handler tests restated
(internal/check/handler_test.go:41-109, internal/expand/handler_test.go:30-108) plus the
batch-check endpoint.  URL parsing and expand run on CPU; check routes need the GPU."""
import json

import pytest

from keto_amd import _lib as L
from keto_amd import check, expand
from keto_amd import relationtuple as rt
from keto_amd.handler import BadRequest, Handler, go_parse_int, relation_query_from_url, tuple_from_json, tuple_from_url
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


def test_json_tuple_rejects_non_string_fields():
    """encoding/json into string fields: numbers, bools, lists are a 400, null is "" """
    for bad in ({"namespace": "n", "object": 1, "relation": "r", "subject_id": "s"},
                {"namespace": "n", "object": "o", "relation": "r", "subject_id": 7},
                {"namespace": "n", "object": "o", "relation": "r", "subject_set": "n:o#r"},
                {"namespace": "n", "object": "o", "relation": "r", "subject_set": {"namespace": ["x"]}},
                {"namespace": True, "object": "o", "relation": "r", "subject_id": "s"}):
        with pytest.raises(BadRequest, match="cannot unmarshal"):
            tuple_from_json(bad)
    t = tuple_from_json({"namespace": "n", "object": None, "relation": "r", "subject_set": {"namespace": "a"}})
    assert t == rt.InternalRelationTuple("n", "", "r", rt.SubjectSet("a", "", ""))
    # *string / *SubjectSet decoding: a key holding null counts as absent (definitions.go:316-325)
    t = tuple_from_json({"namespace": "n", "object": "o", "relation": "r", "subject_id": "u", "subject_set": None})
    assert t == rt.InternalRelationTuple("n", "o", "r", rt.SubjectID("u"))
    with pytest.raises(BadRequest, match="exactly one"):
        tuple_from_json({"namespace": "n", "object": "o", "relation": "r", "subject_id": "u",
                         "subject_set": {"namespace": "a"}})
    h = Handler(None, None)  # both routes answer the type error before any engine call
    assert h.post_check(b'{"namespace":"n","object":1,"relation":"r","subject_id":"s"}')[0] == 400
    assert h.post_check(b'{"namespace":"n","object":"o","relation":"r","subject_set":5}')[0] == 400
    code, body = h.post_check_batch(b'{"tuples":[{"namespace":"n","object":1,"relation":"r","subject_id":"s"}]}')
    assert code == 200 and body["results"][0]["error"]["code"] == 400


def test_max_depth_parses_like_strconv_parseint():
    """strconv.ParseInt(s, 0, 0) of getExpand (internal/expand/handler.go:79)"""
    ok = {"10": 10, "010": 8, "0x1F": 31, "0X1f": 31, "0o17": 15, "0b101": 5, "-3": -3, "+4": 4, "0": 0,
          "1_000": 1000, "0x_1F": 31, "0_7": 7, "9223372036854775807": 2**63 - 1, "-9223372036854775808": -2**63}
    for s, v in ok.items():
        assert go_parse_int(s) == v, s
    for s in ("", " 3", "3 ", "08", "0x", "1__0", "_1", "1_", "0b2", "+-1", "9223372036854775808", "1e3", "٣"):
        with pytest.raises(ValueError):
            go_parse_int(s)
    # a missing max-depth reads as "" (r.URL.Query().Get), quoted like strconv.Quote
    code, body = Handler(None, None).get_expand("namespace=n")
    assert code == 400 and 'parsing ""' in str(body)


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
    # Go base-0 syntax: "02" is octal 2; a depth above int32 is the full tree, not a truncation
    full = h.get_expand("namespace=expand+handler&object=root&relation=parent+of&max-depth=2")[1]
    assert h.get_expand("namespace=expand+handler&object=root&relation=parent+of&max-depth=02")[1] == full
    assert h.get_expand("namespace=expand+handler&object=root&relation=parent+of&max-depth=4294967296")[1] == full
    assert h.get_expand("max-depth=+%203")[0] == 400
    assert h.get_expand("max-depth=99999999999999999999")[0] == 400


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
