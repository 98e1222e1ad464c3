/* Manual API harness: toggle the WebSocket, post Config/Stats, log messages. */
(function () {
  "use strict";
  var n = 0;
  function val(id) { return document.getElementById(id).value; }
  document.addEventListener("DOMContentLoaded", function () {
    document.getElementById("id").value = api.guid();
    document.getElementById("viz").value = api.guid();
    document.getElementById("websocket").addEventListener("click", function (ev) {
      if (ev.target.checked) api.websocketOn(); else api.websocketOff();
    });
    document.getElementById("config").addEventListener("submit", function (ev) {
      ev.preventDefault(); api.postConfig(val("id"), val("host"), val("viz"));
    });
    document.getElementById("stats").addEventListener("submit", function (ev) {
      ev.preventDefault();
      api.postStats(val("count"), val("batch"), val("mse"), val("realStddev"), val("predStddev"));
    });
  });
  api.bind(function (json) {
    var tr = document.createElement("tr");
    [String(++n), String(new Date()), JSON.stringify(json)].forEach(function (t) {
      var td = document.createElement("td"); td.textContent = t; tr.appendChild(td);
    });
    var tb = document.querySelector("table.log tbody");
    tb.insertBefore(tr, tb.firstChild);
  });
})();
