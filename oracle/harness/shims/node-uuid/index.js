// TEST INFRASTRUCTURE ONLY: stand-in for npm node-uuid.  Update ids are
// log-only in the hot path (lib/membership.js:332, lib/dissemination.js:169),
// so a deterministic counter keeps harness runs reproducible.
'use strict';
var n = 0;
module.exports = { v4: function v4() { n += 1; return 'u' + n; }, _reset: function () { n = 0; } };
