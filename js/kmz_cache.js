"use strict";
/*
 * kmz_cache.js -- the cache layer's cross-window merges in columnar form, in
 * Node (SURVEY.md 8f row 2; the Python twin is kmamiz_amd/cache.py).
 *
 * Every realtime tick the reference merges the window into two caches:
 *   new EndpointDependencies(existingDep).combineWith(newDep)
 *                                      RealtimeWorkerImpl.ts:67-70,
 *                                      EndpointDependencies.ts:499-542
 *   CEndpointDependencies.setData  ->  trim()   Cacheable/CEndpointDependencies.ts:46-48
 *   CCombinedRealtimeData.setData  ->  filter(rl.service), cached.combineWith(update)
 *                                      Cacheable/CCombinedRealtimeData.ts:47-53,
 *                                      CombinedRealtimeDataList.ts:183-332
 * Here the window side comes straight from the engine as typed arrays: the
 * reduced graph in its exact entry order (kmz_get_dep_entries, the addon's
 * depEntries) and the dense (endpoint x status) groups (kmz_get_groups).  No
 * object per span, per window row or per entry is built; the merged state is
 * columns over an append-only registry of endpoint names and endpoint-info
 * field sets, and toJSON() builds the cache's objects (<= one row per
 * endpoint / per endpoint x status).
 *
 * Node 12 compatible (no ?. / ??).
 */

const INT64_MIN = -(2n ** 63n);

// a field set (an endpoint info without its timestamp) as a map key; an
// absent value (undefined) differs from every present one
function freeze(f) {
  return JSON.stringify(Object.keys(f).sort().map((k) => [k, f[k] === undefined ? { u: 1 } : f[k]]));
}

function strip(o) {
  const r = {};
  for (const k of Object.keys(o)) if (o[k] !== undefined) r[k] = o[k];
  return r;
}

// uniqueEndpointName -> stable id; interned endpoint-info field sets.  Append
// only: every state built on one registry shares its ids.
class Registry {
  constructor() {
    this.names = [];
    this.index = new Map();
    this.infos = [];
    this.infoIndex = new Map();
    this.byObj = new WeakMap();  // long-lived field objects (per-shape identities) -> info id
  }
  nameId(n) {
    let i = this.index.get(n);
    if (i === undefined) {
      i = this.names.length;
      this.index.set(n, i);
      this.names.push(n);
    }
    return i;
  }
  infoId(f) {
    const k = freeze(f);
    let i = this.infoIndex.get(k);
    if (i === undefined) {
      i = this.infos.length;
      this.infoIndex.set(k, i);
      this.infos.push(Object.assign({}, f));
    }
    return i;
  }
  infoOfObj(f) {
    let i = this.byObj.get(f);
    if (i === undefined) {
      i = this.infoId(f);
      this.byObj.set(f, i);
    }
    return i;
  }
}

// ---- the constructor's deprecation filter (EndpointDependencies.ts:20-74) ----------
// EndpointDependencies.parseThresholdToMilliseconds (20-31)
function parseThresholdToMilliseconds(s) {
  if (!s) return 0;
  const m = s.match(/(?:(\d+)d)?(?:(\d+)h)?(?:(\d+)m)?/);
  if (!m) return 0;
  const d = m[1] ? parseInt(m[1], 10) : 0, h = m[2] ? parseInt(m[2], 10) : 0, mi = m[3] ? parseInt(m[3], 10) : 0;
  return ((d * 86400) + (h * 3600) + (mi * 60)) * 1000;
}
// the class's static threshold, parsed once at load from GlobalSettings'
// DEPRECATED_ENDPOINT_THRESHOLD (GlobalSettings.ts:79, EndpointDependencies.ts:33-36)
const deprecation = { ms: parseThresholdToMilliseconds(process.env.DEPRECATED_ENDPOINT_THRESHOLD || "") };
function setDeprecatedThreshold(s) {
  deprecation.ms = parseThresholdToMilliseconds(s || "");
}
// now - threshold, or 0 (no filter) -- taken when an EndpointDependencies is built (49-54)
function deprecatedCutoff() {
  return deprecation.ms === 0 ? 0 : Date.now() - deprecation.ms;
}
// filterOutDeprecatedEndpoint (44-74) over TEndpointDependency objects; like
// the TS it assigns the filtered lists into the rows it keeps
function filterOutDeprecatedRows(rows, cutoff) {
  if (cutoff === undefined) cutoff = deprecatedCutoff();
  if (cutoff === 0) return rows;
  const gone = new Set();
  const kept = rows.filter((d) => {
    if (d.lastUsageTimestamp < cutoff) {
      gone.add(d.endpoint.uniqueEndpointName);
      return false;
    }
    return true;
  });
  for (const d of kept) {
    d.dependingBy = d.dependingBy.filter((x) => !gone.has(x.endpoint.uniqueEndpointName));
    d.dependingOn = d.dependingOn.filter((x) => !gone.has(x.endpoint.uniqueEndpointName));
  }
  return kept;
}

// Reduced EndpointDependencies: one merged row per endpoint.  Rows (in row
// order): rowEp (registry id), rowInfo / rowTs (the row's `endpoint`), rowLast
// (lastUsageTimestamp), rowExt (isDependedByExternal).  Entries: eRow (the
// row's endpoint), eSide (0 dependingBy, 1 dependingOn), eEp / eDist (the
// entry's endpoint and distance), eInfo / eTs (its endpoint info), and its
// place in the row's list (eHi, eLo): increasing lexicographically.
class ReducedDependencies {
  constructor(reg) {
    this.reg = reg || new Registry();
    this.rowEp = [];
    this.rowInfo = [];
    this.rowTs = [];
    this.rowLast = [];
    this.rowExt = [];
    this.eRow = [];
    this.eSide = [];
    this.eEp = [];
    this.eDist = [];
    this.eInfo = [];
    this.eTs = [];
    this.eHi = [];
    this.eLo = [];
    this.nextHi = 0;
  }

  // The engine's reduced graph of one window (EndpointDependencies([])
  // .combineWith(traces.toEndpointDependencies()).trim()): `dep` from the
  // addon's depEntries, `endpoints` its kmz_endpoint records (24 B each),
  // names[e] the uniqueEndpointName of window endpoint e, shapeFields(s) the
  // ToEndpointInfo fields of shape s (Traces.ts:213-241).
  static fromWindow(dep, endpoints, names, shapeFields, reg) {
    const out = new ReducedDependencies(reg);
    const R = out.reg;
    const emap = names.map((n) => (n === null || n === undefined ? -1 : R.nameId(n)));
    const ep = endpoints instanceof DataView ? endpoints : new DataView(endpoints);
    const E = names.length;
    const rows = [];
    for (let e = 0; e < E; e++) if (ep.getUint32(e * 24 + 20, true)) rows.push(e);
    const first = rows.map((e) => ep.getBigUint64(e * 24 + 8, true));
    const order = rows.map((_, i) => i).sort((a, b) => (first[a] < first[b] ? -1 : first[a] > first[b] ? 1 : 0));
    const infoOfShape = new Map();
    const infoOf = (s) => {
      let i = infoOfShape.get(s);
      if (i === undefined) {
        i = R.infoOfObj(shapeFields(s));
        infoOfShape.set(s, i);
      }
      return i;
    };
    for (const k of order) {
      const e = rows[k];
      const last = ep.getBigInt64(e * 24, true);
      out.rowEp.push(emap[e]);
      out.rowInfo.push(infoOf(dep.rowShape[e]));
      out.rowTs.push(Number(dep.rowTs[e]) / 1000);
      out.rowLast.push(last === INT64_MIN ? 0 : Math.max(0, Number(last) / 1000));
      out.rowExt.push(ep.getUint32(e * 24 + 16, true) !== 0);
    }
    const v = new DataView(dep.entries);
    let maxHi = -1;
    for (let j = 0; j < dep.n; j++) {
      const o = j * 48;
      const lo32 = v.getUint32(o, true), hi32 = v.getUint32(o + 4, true);
      const side = lo32 & 1, dist = (lo32 >>> 1) & 0x7fff;
      const desc = (lo32 >>> 16) | ((hi32 & 0xff) << 16), anc = hi32 >>> 8;
      const row = Number(v.getBigUint64(o + 8, true));
      out.eRow.push(emap[side ? anc : desc]);
      out.eEp.push(emap[side ? desc : anc]);
      out.eSide.push(side);
      out.eDist.push(dist);
      out.eInfo.push(infoOf(v.getUint32(o + 40, true)));
      out.eTs.push(Number(v.getBigInt64(o + 32, true)) / 1000);
      // within a merged row: the contributing row, then its own order (side 1:
      // the first descendant's index, lowerMap order; side 0: the distance)
      out.eHi.push(row);
      out.eLo.push(side ? Number(v.getBigUint64(o + 24, true)) : dist);
      if (row > maxHi) maxHi = row;
    }
    out.nextHi = maxHi + 1;
    return out.filtered();  // (every EndpointDependencies built on the way filters)
  }

  // Columns of TEndpointDependency objects (the cache's JSON).  mergeRows
  // false reads them as `this` of combineWith (a later row of an endpoint
  // replaces an earlier one at its position: Map.set, EndpointDependencies.ts:
  // 508-513), true as its argument (later rows append their unseen entries,
  // 514-535).  Each row's lists are deduplicated as trim() does.
  static fromJSON(rows, mergeRows, reg) {
    const out = new ReducedDependencies(reg);
    const R = out.reg;
    const order = [];
    const byEp = new Map();
    rows = filterOutDeprecatedRows(rows.slice());  // new EndpointDependencies(rows)
    const lists = (r) =>
      ["dependingBy", "dependingOn"].map((lk) => {
        const seen = new Map(), lst = [];
        for (const x of r[lk]) {
          const kk = `${x.endpoint.uniqueEndpointName}\t${x.distance}`;
          if (seen.has(kk)) lst[seen.get(kk)][1] = x;
          else {
            seen.set(kk, lst.length);
            lst.push([kk, x]);
          }
        }
        return lst;
      });
    for (const r of rows) {
      const e = R.nameId(r.endpoint.uniqueEndpointName);
      const ls = lists(r);
      if (!byEp.has(e)) {
        order.push(e);
        byEp.set(e, { r, ls, sets: ls.map((l) => new Set(l.map((p) => p[0]))) });
      } else if (!mergeRows) {
        byEp.set(e, { r, ls, sets: ls.map((l) => new Set(l.map((p) => p[0]))) });
      } else {
        const slot = byEp.get(e);
        for (let side = 0; side < 2; side++)
          for (const p of ls[side])
            if (!slot.sets[side].has(p[0])) {
              slot.sets[side].add(p[0]);
              slot.ls[side].push(p);
            }
      }
    }
    const noTs = (f) => {
      const c = Object.assign({}, f);
      delete c.timestamp;
      return c;
    };
    let ord = 0;
    for (const e of order) {
      const { r, ls } = byEp.get(e);
      out.rowEp.push(e);
      out.rowInfo.push(R.infoId(noTs(r.endpoint)));
      out.rowTs.push(r.endpoint.timestamp);
      out.rowLast.push(r.lastUsageTimestamp);
      out.rowExt.push(!!r.isDependedByExternal);
      for (let side = 0; side < 2; side++)
        for (const [, x] of ls[side]) {
          out.eRow.push(e);
          out.eSide.push(side);
          out.eEp.push(R.nameId(x.endpoint.uniqueEndpointName));
          out.eDist.push(Number(x.distance));
          out.eInfo.push(R.infoId(noTs(x.endpoint)));
          out.eTs.push(x.endpoint.timestamp);
          out.eHi.push(0);
          out.eLo.push(ord++);
        }
    }
    out.nextHi = 1;
    return mergeRows ? out.filtered() : out;
  }

  // the constructor's deprecation filter (EndpointDependencies.ts:44-74) on the
  // columns: rows used before the cutoff go, with every entry naming them
  filtered(cutoff) {
    if (cutoff === undefined) cutoff = deprecatedCutoff();
    if (cutoff === 0) return this;
    const gone = new Set();
    this.rowEp.forEach((e, k) => {
      if (this.rowLast[k] < cutoff) gone.add(e);
    });
    if (gone.size === 0) return this;
    const out = new ReducedDependencies(this.reg);
    const rk = [];
    this.rowEp.forEach((e, k) => {
      if (!gone.has(e)) rk.push(k);
    });
    for (const c of ["rowEp", "rowInfo", "rowTs", "rowLast", "rowExt"]) out[c] = rk.map((k) => this[c][k]);
    const ek = [];
    for (let j = 0; j < this.eRow.length; j++) if (!gone.has(this.eRow[j]) && !gone.has(this.eEp[j])) ek.push(j);
    for (const c of ["eRow", "eSide", "eEp", "eDist", "eInfo", "eTs", "eHi", "eLo"]) out[c] = ek.map((j) => this[c][j]);
    out.nextHi = this.nextHi;
    return out;
  }

  // EndpointDependencies.ts:499-542 on the columns: this's rows keep their
  // place and values (the reference writes the max lastUsageTimestamp into
  // the incoming row object, which it then drops, 516), new endpoints' rows
  // follow in the argument's order, and each row's unseen (name, distance)
  // entries are appended in the argument's order.
  combineWith(other) {
    const out = new ReducedDependencies(this.reg);
    const R = out.reg;
    let bmap = null, imap = null;
    if (other.reg !== R) {
      bmap = other.reg.names.map((n) => R.nameId(n));
      imap = other.reg.infos.map((f) => R.infoId(f));
    }
    const mapE = (x) => (bmap ? bmap[x] : x), mapI = (x) => (imap ? imap[x] : x);
    const have = new Set(this.rowEp);
    const cols = ["rowEp", "rowInfo", "rowTs", "rowLast", "rowExt"];
    for (const c of cols) out[c] = this[c].slice();
    for (let k = 0; k < other.rowEp.length; k++) {
      const e = mapE(other.rowEp[k]);
      if (have.has(e)) continue;
      have.add(e);
      out.rowEp.push(e);
      out.rowInfo.push(mapI(other.rowInfo[k]));
      out.rowTs.push(other.rowTs[k]);
      out.rowLast.push(other.rowLast[k]);
      out.rowExt.push(other.rowExt[k]);
    }
    const ecols = ["eRow", "eSide", "eEp", "eDist", "eInfo", "eTs", "eHi", "eLo"];
    for (const c of ecols) out[c] = this[c].slice();
    // entry identity: (row endpoint, side, endpoint, distance) (distance < 2^15, ids < 2^24)
    const key = (row, side, e, d) => `${row}\t${side}\t${e}\t${d}`;
    const seen = new Set();
    for (let j = 0; j < this.eRow.length; j++) seen.add(key(this.eRow[j], this.eSide[j], this.eEp[j], this.eDist[j]));
    const idx = [];
    for (let j = 0; j < other.eRow.length; j++) idx.push(j);
    idx.sort((a, b) => other.eHi[a] - other.eHi[b] || other.eLo[a] - other.eLo[b]);
    let rank = 0;
    for (const j of idx) {
      const row = mapE(other.eRow[j]), e = mapE(other.eEp[j]);
      const k = key(row, other.eSide[j], e, other.eDist[j]);
      if (seen.has(k)) continue;
      seen.add(k);
      out.eRow.push(row);
      out.eSide.push(other.eSide[j]);
      out.eEp.push(e);
      out.eDist.push(other.eDist[j]);
      out.eInfo.push(mapI(other.eInfo[j]));
      out.eTs.push(other.eTs[j]);
      out.eHi.push(this.nextHi);
      out.eLo.push(rank++);
    }
    out.nextHi = this.nextHi + 1;
    return out.filtered();  // new EndpointDependencies(...) (EndpointDependencies.ts:539-541)
  }

  // EndpointDependencies.ts:91-112: no list dedup needed here (entries are
  // unique per (row, side, name, distance) by construction); the new object's
  // constructor filters deprecated endpoints
  trim() {
    return this.filtered();
  }

  get length() {
    return this.rowEp.length;
  }

  toJSON() {
    const infos = this.reg.infos;
    const info = (i, ts) => strip(Object.assign({}, infos[i], { timestamp: ts }));
    const pos = new Map();
    this.rowEp.forEach((e, k) => pos.set(e, k));
    const idx = [];
    for (let j = 0; j < this.eRow.length; j++) idx.push(j);
    const rp = this.eRow.map((e) => pos.get(e));
    idx.sort((a, b) => rp[a] - rp[b] || this.eSide[a] - this.eSide[b] || this.eHi[a] - this.eHi[b] ||
      this.eLo[a] - this.eLo[b]);
    const out = this.rowEp.map((_, k) => ({
      endpoint: info(this.rowInfo[k], this.rowTs[k]),
      lastUsageTimestamp: this.rowLast[k],
      isDependedByExternal: this.rowExt[k],
      dependingBy: [],
      dependingOn: [],
    }));
    for (const j of idx) {
      const x = { endpoint: info(this.eInfo[j], this.eTs[j]), distance: this.eDist[j],
                  type: this.eSide[j] ? "SERVER" : "CLIENT" };
      (this.eSide[j] ? out[rp[j]].dependingOn : out[rp[j]].dependingBy).push(x);
    }
    return out;
  }
}

// EndpointDependencies.trim() (EndpointDependencies.ts:91-112) over plain
// TEndpointDependency rows (the first tick's per-row graph): each list
// deduplicated by `distance\tname`, first position, last value
function trimRows(rows) {
  const dedup = (lst) => {
    const m = new Map();
    for (const x of lst) m.set(`${x.distance}\t${x.endpoint.uniqueEndpointName}`, x);
    return [...m.values()];
  };
  return filterOutDeprecatedRows(
    rows.map((d) => Object.assign({}, d, { dependingBy: dedup(d.dependingBy), dependingOn: dedup(d.dependingOn) })));
}

// RealtimeWorkerImpl.ts:67-70: existingDep ? new EndpointDependencies(existingDep).combineWith(newDep) : newDep
function workerDependencies(existing, win) {
  return existing ? existing.combineWith(win) : win;
}

// Cacheable/CEndpointDependencies.ts:46-48 (no Mongo)
class CEndpointDependencies {
  constructor(init) {
    this._data = init || null;
  }
  setData(update) {
    this._data = update.trim();
  }
  getData() {
    return this._data;
  }
}

// ---- combined realtime data ----------------------------------------------------
const BASE = ["uniqueServiceName", "service", "namespace", "version", "method", "requestContentType",
              "responseContentType"];
const BODY = ["requestBody", "requestSchema", "responseBody", "responseSchema"];

// Utils.ToPrecise (Utils.ts:311-313)
function toPrecise(x) {
  return Math.round((x + Number.EPSILON) * 1e14) / 1e14;
}

// CombinedRealtimeDataList.ts:278-332, the reference's operations in its order
function combineLatencyCVAndMean(n1, mean1, cv1, n2, mean2, cv2) {
  const safeLog10 = (x) => (x <= 0 ? 0 : Math.floor(Math.log10(x)));
  const shift = Math.floor((safeLog10(mean1) + safeLog10(mean2)) / 2);
  const scale = Math.pow(10, shift);
  const mean1s = mean1 / scale, mean2s = mean2 / scale;
  const std1s = cv1 * mean1s, std2s = cv2 * mean2s;
  const totalN = n1 + n2;
  const meanTotal = (n1 * mean1s + n2 * mean2s) / totalN;
  const variance1 = std1s ** 2, variance2 = std2s ** 2;
  const pooledVariance = (n1 * variance1 + n2 * variance2 + n1 * (mean1s - meanTotal) ** 2 +
    n2 * (mean2s - meanTotal) ** 2) / totalN;
  const stdTotal = Math.sqrt(pooledVariance);
  return { mean: meanTotal * scale, cv: meanTotal === 0 ? 0 : stdTotal / meanTotal };
}

// CombinedRealtimeDataList as columns: one row per (endpoint, status); `key`
// the interned `uniqueEndpointName\tstatus`, `meta` the row's sample fields.
class CombinedColumns {
  constructor(tab) {
    this.tab = tab || { keys: new Map(), metas: [], metaIndex: new Map() };
    this.key = [];
    this.meta = [];
    this.combined = [];
    this.latest = [];
    this.mean = [];
    this.cv = [];
    this.body = { requestBody: [], requestSchema: [], responseBody: [], responseSchema: [] };
  }
  _keyId(k) {
    let i = this.tab.keys.get(k);
    if (i === undefined) {
      i = this.tab.keys.size;
      this.tab.keys.set(k, i);
    }
    return i;
  }
  _metaId(m) {
    const f = freeze(m);
    let i = this.tab.metaIndex.get(f);
    if (i === undefined) {
      i = this.tab.metas.length;
      this.tab.metaIndex.set(f, i);
      this.tab.metas.push(m);
    }
    return i;
  }
  _push(m, combined, latest, mean, cv, bodies) {
    this.key.push(this._keyId(`${m.uniqueEndpointName}\t${m.status}`));
    this.meta.push(this._metaId(m));
    this.combined.push(combined);
    this.latest.push(latest);
    this.mean.push(mean);
    this.cv.push(cv);
    for (const f of BODY) this.body[f].push(bodies ? bodies[f] : undefined);
  }
  static fromJSON(rows, like) {
    const out = new CombinedColumns(like ? like.tab : null);
    for (const r of rows) {
      const m = { uniqueEndpointName: r.uniqueEndpointName, status: r.status };
      for (const b of BASE) m[b] = r[b];
      out._push(m, r.combined, r.latestTimestamp, r.latency.mean, r.latency.cv, r);
    }
    return out;
  }
  // RealtimeDataList.toCombinedRealtimeData() straight from the engine's
  // dense groups (kmz_group, 40 B; [n_ep * n_status]): used groups ordered by
  // their endpoint's first row, then their own first row
  // (RealtimeDataList.ts:22-45).  epFields(e): the row fields of endpoint e;
  // statuses[s]: the status strings.  No Envoy logs (no content types).
  static fromGroups(groups, nStatus, epFields, statuses, like) {
    const out = new CombinedColumns(like ? like.tab : null);
    const v = groups instanceof DataView ? groups : new DataView(groups);
    const G = v.byteLength / 40;
    const used = [], epFirst = new Map();
    for (let g = 0; g < G; g++) {
      const n = v.getBigUint64(g * 40, true);
      if (!n) continue;
      const first = v.getBigUint64(g * 40 + 8, true), e = Math.floor(g / nStatus);
      if (!epFirst.has(e) || first < epFirst.get(e)) epFirst.set(e, first);
      used.push({ g, e, n: Number(n), first });
    }
    const cmp = (a, b) => (a < b ? -1 : a > b ? 1 : 0);
    used.sort((a, b) => cmp(epFirst.get(a.e), epFirst.get(b.e)) || cmp(a.first, b.first));
    for (const { g, e, n } of used) {
      const f = epFields(e);
      const m = { uniqueEndpointName: f.uniqueEndpointName, status: statuses[g % nStatus] };
      for (const b of BASE) m[b] = f[b];
      out._push(m, n, Number(v.getBigInt64(g * 40 + 16, true)), v.getFloat64(g * 40 + 24, true),
                v.getFloat64(g * 40 + 32, true), null);
    }
    return out;
  }
  _take(sel) {
    const out = new CombinedColumns(this.tab);
    for (let j = 0; j < this.key.length; j++) {
      if (!sel(j)) continue;
      for (const c of ["key", "meta", "combined", "latest", "mean", "cv"]) out[c].push(this[c][j]);
      for (const f of BODY) out.body[f].push(this.body[f][j]);
    }
    return out;
  }
  // update.toJSON().filter((rl) => rl.service) (CCombinedRealtimeData.ts:48-50)
  filterService() {
    return this._take((j) => !!this.tab.metas[this.meta[j]].service);
  }
  filterNamespace(ns) {
    return this._take((j) => this.tab.metas[this.meta[j]].namespace === ns);
  }
  // CombinedRealtimeDataList.ts:183-263: groups in first-appearance order of
  // this + other; the sample is the group's first row; timestamps by
  // Math.max; bodies by Utils.Merge with their schemas re-derived; the latency
  // fold from (0, 0, 0) in list order, then ToPrecise.
  combineWith(other, merge, toSchema) {
    const out = new CombinedColumns(this.tab);
    const rows = [];  // [source, index]
    for (let j = 0; j < this.key.length; j++) rows.push([this, j]);
    for (let j = 0; j < other.key.length; j++) rows.push([other, j]);
    const groups = new Map();
    for (const [src, j] of rows) {
      const m = src.tab.metas[src.meta[j]];
      const id = `${m.uniqueEndpointName}\t${m.status}`;
      if (!groups.has(id)) groups.set(id, []);
      groups.get(id).push([src, j]);
    }
    for (const grp of groups.values()) {
      const [s0, j0] = grp[0];
      const m = s0.tab.metas[s0.meta[j0]];
      let combined = 0;
      for (const [s, j] of grp) combined += s.combined[j];
      let latest = s0.latest[j0];
      const b = {};
      for (const f of BODY) b[f] = s0.body[f][j0];
      for (let k = 1; k < grp.length; k++) {
        const [s, j] = grp[k];
        latest = Math.max(latest, s.latest[j]);
        if (merge) {
          b.requestBody = merge(b.requestBody, s.body.requestBody[j]);
          b.responseBody = merge(b.responseBody, s.body.responseBody[j]);
          if (b.requestBody) b.requestSchema = toSchema(b.requestBody);
          if (b.responseBody) b.responseSchema = toSchema(b.responseBody);
        }
      }
      let acc = { mean: 0, cv: 0, n: 0 };
      for (const [s, j] of grp) {
        const r = combineLatencyCVAndMean(acc.n, acc.mean, acc.cv, s.combined[j], s.mean[j], s.cv[j]);
        acc = { mean: r.mean, cv: r.cv, n: acc.n + s.combined[j] };
      }
      out._push(m, combined, latest, toPrecise(acc.mean), toPrecise(acc.cv), b);
    }
    return out;
  }
  get length() {
    return this.key.length;
  }
  toJSON() {
    return this.key.map((_, j) => {
      const m = this.tab.metas[this.meta[j]];
      return strip({
        uniqueEndpointName: m.uniqueEndpointName,
        uniqueServiceName: m.uniqueServiceName,
        service: m.service,
        namespace: m.namespace,
        version: m.version,
        method: m.method,
        status: m.status,
        combined: this.combined[j],
        requestContentType: m.requestContentType,
        responseContentType: m.responseContentType,
        latestTimestamp: this.latest[j],
        requestBody: this.body.requestBody[j],
        requestSchema: this.body.requestSchema[j],
        responseBody: this.body.responseBody[j],
        responseSchema: this.body.responseSchema[j],
        latency: { mean: this.mean[j], cv: this.cv[j] },
      });
    });
  }
}

// Cacheable/CCombinedRealtimeData.ts:47-53 (no Mongo)
class CCombinedRealtimeData {
  constructor(init, merge, toSchema) {
    this._data = init || null;
    this._merge = merge;
    this._toSchema = toSchema;
  }
  setData(update) {
    update = update.filterService();
    this._data = this._data ? this._data.combineWith(update, this._merge, this._toSchema) : update;
  }
  getData(namespace) {
    return namespace && this._data ? this._data.filterNamespace(namespace) : this._data;
  }
}

module.exports = { Registry, ReducedDependencies, CombinedColumns, CEndpointDependencies, CCombinedRealtimeData,
                   workerDependencies, combineLatencyCVAndMean, toPrecise, trimRows, parseThresholdToMilliseconds,
                   setDeprecatedThreshold, deprecatedCutoff, filterOutDeprecatedRows };
