module.exports = require('./typed.js');
