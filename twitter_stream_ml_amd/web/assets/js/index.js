/* Dashboard: Config messages rebuild the embedded Lightning plots and reset
 * the counters; Stats messages update the counters. */
(function () {
  "use strict";
  var FIELDS = ["count", "batch", "mse", "realStddev", "predStddev"];
  function set(id, v) { document.getElementById(id).textContent = v; }

  function onConfig(json) {
    var graphs = document.getElementById("graphs");
    graphs.innerHTML = "";
    FIELDS.forEach(function (f) { set(f, "0"); });
    if (!json.id || json.host === "") return;
    (json.viz || []).forEach(function (vizId) {
      var div = document.createElement("div");
      div.id = "graph" + vizId;
      graphs.appendChild(div);
      new embed.Parent(div.id, json.host + "/visualizations/" + vizId + "/pym");
    });
  }

  function onStats(json) { FIELDS.forEach(function (f) { set(f, json[f]); }); }

  api.bind(function (json) {
    if (json.jsonClass === "Config") onConfig(json);
    else if (json.jsonClass === "Stats") onStats(json);
  });
  api.onState = function (up) {
    var c = document.getElementById("conn");
    c.textContent = up ? "live" : "offline";
    c.className = "conn " + (up ? "on" : "off");
  };
  document.addEventListener("DOMContentLoaded", function () {
    api.getStats();
    api.websocketOn();
  });
})();
