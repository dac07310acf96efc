// TEST INFRASTRUCTURE ONLY: forwards to node's stream module.
'use strict';
module.exports = require('stream');
