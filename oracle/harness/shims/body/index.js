// TEST INFRASTRUCTURE ONLY: request forwarding is out of scope.
'use strict';
module.exports = function body(req, res, opts, cb) { (cb || opts)(null, ''); };
