/* twtml-web client API (behaviour of the reference's api.js, dependency-free):
 * a WebSocket on /api that reconnects every 5 s, GET /api/{config,stats},
 * and posts of {"jsonClass": "Config"|"Stats", ...} over the socket when it
 * is open, else HTTP POST /api followed by a GET refresh. */
(function (global) {
  "use strict";
  var listeners = [];
  var api = { socket: null, wanted: false, reconnectMs: 5000 };

  api.bind = function (cb) { listeners.push(cb); };
  api.onMessage = function (json) { listeners.forEach(function (cb) { cb(json); }); };
  api.onState = function () {};

  function wsUrl() {
    var l = global.location;
    return (l.protocol === "https:" ? "wss://" : "ws://") + l.host + "/api";
  }

  api.websocketOn = function () {
    api.wanted = true;
    if (api.socket) return;
    var ws = new WebSocket(wsUrl());
    api.socket = ws;
    ws.onopen = function () { api.onState(true); };
    ws.onmessage = function (ev) {
      try { api.onMessage(JSON.parse(ev.data)); } catch (e) { console.log("bad json", ev.data); }
    };
    ws.onclose = function () {
      api.socket = null; api.onState(false);
      if (api.wanted) setTimeout(api.websocketOn, api.reconnectMs);
    };
  };

  api.websocketOff = function () {
    api.wanted = false;
    if (api.socket) { api.socket.close(); api.socket = null; }
  };

  api.get = function (kind) {
    return fetch("/api/" + kind, { headers: { accept: "application/json" } })
      .then(function (r) { return r.json(); }).then(api.onMessage);
  };
  api.getConfig = function () { return api.get("config"); };
  api.getStats = function () { return api.get("stats"); };

  api.post = function (json, kind) {
    var str = JSON.stringify(json);
    if (api.socket && api.socket.readyState === 1) { api.socket.send(str); return Promise.resolve(); }
    return fetch("/api", { method: "POST", body: str,
                           headers: { "content-type": "application/json" } })
      .then(function () { return api.get(kind); });
  };

  api.postConfig = function (id, host, viz) {
    return api.post({ jsonClass: "Config", id: id, host: host,
                      viz: Array.isArray(viz) ? viz : [viz] }, "config");
  };

  api.postStats = function (count, batch, mse, realStddev, predStddev) {
    return api.post({ jsonClass: "Stats", count: parseInt(count, 10), batch: parseInt(batch, 10),
                      mse: parseInt(mse, 10), realStddev: parseInt(realStddev, 10),
                      predStddev: parseInt(predStddev, 10) }, "stats");
  };

  api.guid = function () {
    function s4() { return Math.floor((1 + Math.random()) * 0x10000).toString(16).substring(1); }
    return s4() + s4() + "-" + s4() + "-" + s4() + "-" + s4() + "-" + s4() + s4() + s4();
  };

  global.api = api;
})(window);
