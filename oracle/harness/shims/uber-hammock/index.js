// TEST INFRASTRUCTURE ONLY: request forwarding is out of scope.
'use strict';
module.exports = { Request: function () {}, Response: function () {} };
