// TEST INFRASTRUCTURE ONLY: stand-in for npm error/typed.
'use strict';
module.exports = function TypedError(spec) {
    return function create(fields) {
        var msg = String(spec.message || '').replace(/\{(\w+)\}/g, function (_, k) {
            return fields && k in fields ? String(fields[k]) : '';
        });
        var e = new Error(msg);
        Object.keys(spec).forEach(function (k) { if (k !== 'message') e[k] = spec[k]; });
        if (fields) Object.keys(fields).forEach(function (k) { e[k] = fields[k]; });
        e.type = spec.type;
        return e;
    };
};
