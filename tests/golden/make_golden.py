#!/usr/bin/env python3
"""Regenerate tests/golden/known_answers.json from the reference's own tests.

Run in the build container only (reads /root/reference, which does not exist on
the GPU box). The output is DATA: the expected inputs/outputs the reference's
tests assert, transcribed as JSON vectors. No reference source travels.

Sources (reference checkout, Grafana Tempo ~v1.4.1):
  * tempodb/encoding/v2/backend_block_test.go:14-85   TestV2Block ids + objects
    for the committed v2test block (copied as data to tests/golden/v2test/).
  * pkg/tempofb/searchdata_test.go:95-124            TestContainsTag table
  * tempodb/search/pipeline_test.go:15-282           TestPipelineMatches* tables
  * tempodb/search/backend_search_block_test.go:24-88 TestBackendSearchBlockSearch
  * tempodb/search/streaming_search_block_test.go:101-154 metrics expectations
  * tempodb/encoding/common/bloom_test.go:120-154    TestBloomShardCount clamps
  * modules/ingester/instance_search_test.go:41-97,331-371 TestInstanceSearch /
    TestInstanceSearchMetrics live-trace stage (parsed: trace counts, tag, fraction)
The pipeline tables use time.Now()-relative timestamps in Go; they are pinned
here at a fixed NOW so the vectors are reproducible (the predicates only depend
on differences and second truncation, which the chosen NOW keeps identical).
"""
import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def parse_byte_slices(block):
    out = []
    for m in re.finditer(r"\{([0-9a-fx,\s]+)\}", block):
        vals = [v.strip() for v in m.group(1).split(",") if v.strip()]
        out.append(bytes(int(v, 16) for v in vals).hex())
    return out


def v2test_vectors():
    src = open(os.path.join(REF, "tempodb/encoding/v2/backend_block_test.go")).read()
    ids_block = src[src.index("ids := [][]byte{"): src.index("// objs")]
    objs_block = src[src.index("objs := [][]byte{"): src.index("meta := backend.NewBlockMeta")]
    ids = parse_byte_slices(ids_block.split("{", 1)[1])
    objs = parse_byte_slices(objs_block.split("{", 1)[1])
    assert len(ids) == 10 and len(objs) == 10, (len(ids), len(objs))
    return {"block_id": "4cd3c468-6398-481b-b5ec-de56d1048427", "ids": ids, "objs": objs,
            # verified properties: index page checksum, records
            "index_checksum": "8225cdc5ec7a0856", "total_records": 2}


NOW_NS = 1_700_000_000_123_456_789  # fixed "time.Now()" for the pipeline tables
SEC = 1_000_000_000
MS = 1_000_000
MIN = 60 * SEC


def unix(ns):
    return ns // SEC


def pipeline_tables():
    # TestPipelineMatchesTags (pipeline_test.go:15-80)
    tags = [
        {"name": "match", "data": {"key": ["value"]}, "req": {"key": "value"}, "match": True},
        {"name": "noMatch", "data": {"key1": ["value"]}, "req": {"key2": "value"}, "match": False},
        {"name": "matchSubstring", "data": {"key": ["avalue"]}, "req": {"key": "val"}, "match": True},
        {"name": "matchMulti", "data": {"key1": ["value1"], "key2": ["value2"], "key3": ["value3"], "key4": ["value4"]},
         "req": {"key1": "value1", "key3": "value3"}, "match": True},
        {"name": "noMatchMulti", "data": {"key1": ["value1"], "key2": ["value2"]},
         "req": {"key1": "value1", "key3": "value3"}, "match": False},
        {"name": "rewriteError", "data": {"status.code": ["2"]}, "req": {"error": "true"}, "match": True},
        {"name": "rewriteStatusCode", "data": {"status.code": ["2"]}, "req": {"status.code": "error"}, "match": True},
    ]
    n = NOW_NS
    # TestPipelineMatchesTraceDuration (pipeline_test.go:82-150)
    dur = [
        {"name": "no filtering", "start": n, "end": n, "min": 0, "max": 0, "match": True},
        {"name": "match both filters", "start": n, "end": n + 50 * MS, "min": 10, "max": 100, "match": True},
        {"name": "no match either filter", "start": n, "end": n + 200 * MS, "min": 10, "max": 100, "match": False},
        {"name": "match more than 32-bits of nanoseconds", "start": n, "end": n + MIN, "min": 30000, "max": 90000,
         "match": True},
        {"name": "no match more than 32-bits of nanoseconds", "start": n, "end": n + 15 * SEC, "min": 30000,
         "max": 90000, "match": False},
    ]
    # TestPipelineMatchesTraceStartEnd (pipeline_test.go:152-232)
    se = [
        {"name": "no filtering", "start": n, "end": n, "rs": 0, "re": 0, "match": True},
        {"name": "requested range is before span", "start": n - MIN, "end": n - MIN,
         "rs": unix(n - 3 * MIN), "re": unix(n - 2 * MIN), "match": False},
        {"name": "requested range is after span", "start": n - MIN, "end": n - MIN,
         "rs": unix(n - 30 * SEC), "re": unix(n), "match": False},
        {"name": "requested range encloses span", "start": n - MIN, "end": n - MIN,
         "rs": unix(n - 2 * MIN), "re": unix(n), "match": True},
        {"name": "span encloses requested range", "start": n - 2 * MIN, "end": n,
         "rs": unix(n - MIN), "re": unix(n - MIN), "match": True},
        {"name": "range overlaps span start", "start": n - 3 * MIN, "end": n - MIN,
         "rs": unix(n - 4 * MIN), "re": unix(n - 2 * MIN), "match": True},
        {"name": "range overlaps span end", "start": n - 3 * MIN, "end": n - MIN,
         "rs": unix(n - 2 * MIN), "re": unix(n), "match": True},
    ]
    # TestPipelineMatchesBlock (pipeline_test.go:234-282): header tag=value, min 1s, max 10s
    blk = {
        "header": {"tags": {"tag": ["value"]}, "min_dur_ns": 1 * SEC, "max_dur_ns": 10 * SEC},
        "cases": [
            {"name": "no filters", "req": {}, "min": 0, "max": 0, "match": True},
            {"name": "matches all", "req": {"tag": "value"}, "min": 5000, "max": 6000, "match": True},
            {"name": "no matching tag", "req": {"nomatch": "value"}, "min": 0, "max": 0, "match": False},
            {"name": "no matching min duration", "req": {}, "min": 20000, "max": 0, "match": False},
            {"name": "no matching max duration", "req": {}, "min": 0, "max": 500, "match": False},
        ],
    }
    return {"tags": tags, "duration": dur, "start_end": se, "block": blk}


def contains_tag_table():
    # TestContainsTag (pkg/tempofb/searchdata_test.go:95-124): key1..key6 = "value"
    return {
        "entry": {f"key{i}": ["value"] for i in range(1, 7)},
        "cases": [
            {"key": "key1", "value": "value", "found": True},
            {"key": "key1", "value": "value2", "found": False},
            {"key": "key6", "value": "value", "found": True},
            {"key": "key0", "value": "value", "found": False},
            {"key": "key10", "value": "value", "found": False},
        ],
    }


def instance_search_vectors():
    """The live-trace stage of TestInstanceSearch and TestInstanceSearchMetrics, parsed from
    the test source: trace counts, the annotated fraction and the tag."""
    src = open(os.path.join(REF, "modules/ingester/instance_search_test.go")).read()
    t1 = src[src.index("func TestInstanceSearch(t"): src.index("func TestInstanceSearchNoData")]
    n1 = int(re.search(r"numTraces := (\d+)", t1).group(1))
    frac = int(re.search(r"searchAnnotatedFractionDenominator := (\d+)", t1).group(1))
    key = re.search(r'var tagKey = "([^"]*)"', t1).group(1)
    val = re.search(r'var tagValue = "([^"]*)"', t1).group(1)
    t2 = src[src.index("func TestInstanceSearchMetrics"): src.index("func BenchmarkInstanceSearchUnderLoad")]
    n2 = int(re.search(r"numTraces := uint32\((\d+)\)", t2).group(1))
    k2, v2 = re.search(r'data.AddTag\("([^"]*)", "([^"]*)"\)', t2).groups()
    return {
        # every `frac`-th of n1 live traces carries search data {key: val}; Search(key=val)
        # returns n1 / frac traces (:95); the others are live traces with no segments
        "search": {"num_traces": n1, "annotated_every": frac, "tag": [key, val], "expected_results": n1 // frac},
        # n2 live traces, one segment each; an exhaustive search inspects every trace and
        # the sum of the segments' lengths (:368-370)
        "metrics": {"num_traces": n2, "tag": [k2, v2], "expected_traces_inspected": n2,
                    "expected_bytes": "sum of len(searchData)"},
    }


# ---- cross-checks of the transcribed tables against the reference's test source -------
# The tables above are typed out; these parsers read the same Go test tables as text and
# main() refuses to write the fixture unless every case agrees (name, inputs, expectation).
GO_CONST = {  # identifiers the tables use, checked against their declarations below
    "trace.StatusCodeTag": ("pkg/model/trace/matches.go", r'StatusCodeTag\s*=\s*"([^"]*)"'),
    "trace.StatusCodeError": ("pkg/model/trace/matches.go", r'StatusCodeError\s*=\s*"([^"]*)"'),
}


def go_const(name):
    if name.startswith('"'):
        return name.strip('"')
    if name == "strconv.Itoa(int(v1.Status_STATUS_CODE_ERROR))":
        src = open(os.path.join(REF, "pkg/tempopb/trace/v1/trace.pb.go")).read()
        return re.search(r"Status_STATUS_CODE_ERROR\s+Status_StatusCode\s*=\s*(\d+)", src).group(1)
    f, pat = GO_CONST[name]
    return re.search(pat, open(os.path.join(REF, f)).read()).group(1)


def go_cases(src, func):
    """The {...} case literals of a table-driven test, as {field: raw Go expression}."""
    body = src[src.index("func " + func + "("):]
    body = body[body.index("}{") + 2: body.index("\n\t}\n")]
    cases = []
    for m in re.finditer(r"\n\t\t\{\n(.*?)\n\t\t\},", body, re.S):
        f = {}
        for line in m.group(1).split("\n"):
            line = line.split("//")[0].strip().rstrip(",")
            if ":" in line:
                k, v = line.split(":", 1)
                f[k.strip()] = v.strip()
        cases.append(f)
    return cases


def go_map(expr):
    """map[string]string{...} / map[string][]string{...} with constant keys and values."""
    inner = expr[expr.index("{") + 1: expr.rindex("}")]
    out = {}
    for m in re.finditer(r'([\w."()]+(?:\([^)]*\)\))?)\s*:\s*(\{[^}]*\}|[\w."]+(?:\([^)]*\)\))?)', inner):
        k, v = go_const(m.group(1)), m.group(2)
        if v.startswith("{"):
            out[k] = [go_const(x.strip()) for x in v[1:-1].split(",") if x.strip()]
        else:
            out[k] = go_const(v)
    return out


def go_dur(expr):
    """time.Duration expressions of the tables: [-][n *] time.Unit."""
    units = {"time.Millisecond": MS, "time.Second": SEC, "time.Minute": MIN}
    e = expr.replace(" ", "")
    sign = -1 if e.startswith("-") else 1
    e = e.lstrip("-")
    if "*" in e:
        n, u = e.split("*")
        return sign * int(n) * units[u]
    return sign * units[e]


def go_time(expr):
    """time.Now()-relative timestamps at the fixed NOW_NS: .UnixNano() or uint32(...Unix())."""
    e = expr.strip()
    secs = e.startswith("uint32(")
    if secs:
        e = e[len("uint32("):-1]
    ns = NOW_NS
    m = re.match(r"time\.Now\(\)\.Add\((.*)\)\.Unix(Nano)?\(\)$", e)
    if m:
        ns += go_dur(m.group(1))
    elif not re.match(r"time\.Now\(\)\.Unix(Nano)?\(\)$", e):
        raise ValueError(expr)
    return unix(ns) if secs else ns


def go_num(expr):
    return int(expr.replace("_", ""))


def check_pipeline_tables(t):
    src = open(os.path.join(REF, "tempodb/search/pipeline_test.go")).read()
    got = [{"name": go_const(c["name"]), "data": go_map(c["searchData"]), "req": go_map(c["request"]),
            "match": c["shouldMatch"] == "true"} for c in go_cases(src, "TestPipelineMatchesTags")]
    assert got == t["tags"], ("TestPipelineMatchesTags", got)
    got = [{"name": go_const(c["name"]), "start": go_time(c["spanStart"]), "end": go_time(c["spanEnd"]),
            "min": go_num(c["minDurationMs"]), "max": go_num(c["maxDurationMs"]), "match": c["shouldMatch"] == "true"}
           for c in go_cases(src, "TestPipelineMatchesTraceDuration")]
    assert got == t["duration"], ("TestPipelineMatchesTraceDuration", got)
    got = [{"name": go_const(c["name"]), "start": go_time(c["spanStart"]), "end": go_time(c["spanEnd"]),
            "rs": go_time(c["reqStart"]) if "reqStart" in c else 0, "re": go_time(c["reqEnd"]) if "reqEnd" in c else 0,
            "match": c["shouldMatch"] == "true"} for c in go_cases(src, "TestPipelineMatchesTraceStartEnd")]
    assert got == t["start_end"], ("TestPipelineMatchesTraceStartEnd", got)
    body = src[src.index("func TestPipelineMatchesBlock("):]
    tag = re.search(r'commonBlock\.AddTag\("([^"]*)", "([^"]*)"\)', body).groups()
    mn = go_dur(re.search(r"MinDur = uint64\((.*)\)", body).group(1))
    mx = go_dur(re.search(r"MaxDur = uint64\((.*)\)", body).group(1))
    hdr = t["block"]["header"]
    assert hdr == {"tags": {tag[0]: [tag[1]]}, "min_dur_ns": mn, "max_dur_ns": mx}, ("block header", hdr)
    got = []
    for c in go_cases(src, "TestPipelineMatchesBlock"):
        req = c.get("request", "&tempopb.SearchRequest{}")
        inner = req[req.index("{") + 1: req.rindex("}")]
        tags = re.search(r"Tags:\s*(map\[string\]string\{[^}]*\})", inner)
        mnm = re.search(r"MinDurationMs:\s*([\d_]+)", inner)
        mxm = re.search(r"MaxDurationMs:\s*([\d_]+)", inner)
        got.append({"name": go_const(c["name"]), "req": go_map(tags.group(1)) if tags else {},
                    "min": go_num(mnm.group(1)) if mnm else 0, "max": go_num(mxm.group(1)) if mxm else 0,
                    "match": c["shouldMatch"] == "true"})
    assert got == t["block"]["cases"], ("TestPipelineMatchesBlock", got)


def check_contains_tag(t):
    src = open(os.path.join(REF, "pkg/tempofb/searchdata_test.go")).read()
    body = src[src.index("func TestContainsTag("):]
    body = body[: body.index("\n}\n")]
    entry = {}
    for k, v in re.findall(r'm\.AddTag\("([^"]*)", "([^"]*)"\)', body):
        entry.setdefault(k, []).append(v)
    cases = [{"key": k, "value": v, "found": f == "true"}
             for k, v, f in re.findall(r'\{"([^"]*)", "([^"]*)", (true|false)\}', body)]
    assert entry == t["entry"] and cases == t["cases"], ("TestContainsTag", entry, cases)


def main():
    out = {
        "_provenance": "transcribed from the reference's tests by tests/golden/make_golden.py",
        "v2test": v2test_vectors(),
        "contains_tag": contains_tag_table(),
        "pipeline": pipeline_tables(),
        # TestBackendSearchBlockSearch (backend_search_block_test.go:24-88)
        "backend_search_block": {"trace_count": 10000, "query": {"key20": "value_B_20"},
                                  "expected_results": 1, "expected_traces_inspected": 10000,
                                  "encodings": ["none", "snappy"]},
        # TestStreamingSearchBlockSearchBlock (streaming_search_block_test.go:101-154), 10 traces
        "search_block_metrics": {"trace_count": 10, "cases": [
            {"name": "matches every trace", "req": {"key1": "value10"}, "results": 10, "blocks_inspected": 1,
             "traces_inspected": 10, "blocks_skipped": 0},
            {"name": "skips block", "req": {"nomatch": "nomatch"}, "results": 0, "blocks_inspected": 0,
             "traces_inspected": 0, "blocks_skipped": 1},
        ]},
        "instance_search_live": instance_search_vectors(),
        # TestBloomShardCount (bloom_test.go:120-154) + ValidateShardCount
        "bloom_shard_count": [
            {"name": "too many shards", "fp": 0.01, "shard_size": 1, "estimated_objects": 100000,
             "expected_shards": 1000},
            {"name": "too few shards", "fp": 0.01, "shard_size": 10, "estimated_objects": 1, "expected_shards": 1},
        ],
    }
    check_pipeline_tables(out["pipeline"])
    check_contains_tag(out["contains_tag"])
    out["_provenance"] += ("; the pipeline and ContainsTag tables are checked case by case against the "
                           "Go test source (check_pipeline_tables, check_contains_tag)")
    path = os.path.join(HERE, "known_answers.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference checkout not present (build container only)")
    main()
