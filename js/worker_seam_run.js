"use strict";
// node js/worker_seam_run.js <Trace[][] json> <workers> <mode: gpu|load>
// Starts <workers> worker_threads running js/realtime_worker.js at once and
// sends each the same batch (objects to half, raw JSON bytes to the other
// half); prints {results: [...]} with every worker's answer (mode gpu), or
// {loaded: n} once every worker has loaded the addon (mode load: no GPU).
const { Worker } = require("worker_threads");
const fs = require("fs");
const path = require("path");
const file = process.argv[2], nw = Number(process.argv[3] || 2), mode = process.argv[4] || "gpu";
const raw = fs.readFileSync(file);
const traces = JSON.parse(raw.toString("utf8"));
const ws = [];
for (let i = 0; i < nw; i++) ws.push(new Worker(path.join(__dirname, "realtime_worker.js"), { workerData: { ready: true } }));
const ready = ws.map((w) => new Promise((res, rej) => { w.once("message", res); w.once("error", rej); }));
Promise.all(ready).then(() => {
  if (mode === "load") {
    // the addon is loaded (and its exports usable) in every worker context
    process.stdout.write(JSON.stringify({ loaded: ws.length }));
    return Promise.all(ws.map((w) => w.terminate()));
  }
  const jobs = ws.map((w, i) => new Promise((res, rej) => {
    w.once("message", res);
    w.once("error", rej);
    w.postMessage(i % 2 ? { uniqueId: i, json: new Uint8Array(raw) } : { uniqueId: i, traces });
  }));
  return Promise.all(jobs).then((results) => {
    process.stdout.write(JSON.stringify({ results }));
    return Promise.all(ws.map((w) => w.terminate()));
  });
}).catch((e) => { process.stderr.write(String(e && e.stack ? e.stack : e)); process.exit(1); });
