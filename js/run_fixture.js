"use strict";
// node js/run_fixture.js <Trace[][] json> -> prints {rl, crl_rt, crl_tag, deps} as JSON
// (driven by tests/test_gpu_node.py; needs a GPU)
const fs = require("fs");
const { NativeTraces } = require("./kmamiz_native");

const traces = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
const t = new NativeTraces(traces, 0);
const reps = [{ uniqueServiceName: "details\tbook\tv1", replicas: 3 }];
const out = {
  rl: t.toRealTimeData().toJSON(),
  crl_rt: t.toRealTimeData(reps).toCombinedRealtimeData(),
  crl_tag: t.combineLogsToRealtimeData([], reps).toCombinedRealtimeData(),
  deps: t.toEndpointDependencies(),
  info: NativeTraces.ToEndpointInfo(traces[0][0] || { name: "a.b.svc.c", tags: { "http.url": "x" }, timestamp: 0 }),
};
process.stdout.write(JSON.stringify(out));
