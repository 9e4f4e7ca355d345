--[[
multigrid-poisson/hip.lua — drop-in GPU solver class for thenumbernine/lua-multigrid-poisson,
backed by libmgpoisson.so (include/mgpoisson.h) through LuaJIT FFI.

It accepts both constructor protocols of the reference:
  * cpu.lua table protocol (cpu.lua:173-216):
        local MG = require 'multigrid-poisson.hip'
        local mg = MG{size=n, maxiter=?, epsilon=?, errorCallback=function(iter, err) ... end, debug=?}
        mg:solve()            -- or mg:step() -> err
  * cpu-raw.lua / gpu.lua positional protocol (cpu-raw.lua:142, 239; gpu.lua:26, 348):
        local mg = MG(size, real)    -- real = 'double' (default) or 'float'
        mg:run()              -- two outer iterations, prints '#iter err'
        mg:twoGrid(h, uPtr, fPtr, L) -- raw real* host buffers of an L x L grid (cpu-raw.lua:186)
  * cpu-gpu.lua protocol (cpu-gpu.lua:55-72): MG(size, real, cpuDepth[, engine]) switches to the
    GPU's one-launch coarse engine at size 2^cpuDepth, or, given an engine with
    engine:twoGrid(h, uPtr, fPtr, L) (e.g. require'multigrid-poisson.cpu-raw'(2^cpuDepth)), hands
    that level's u and f to it and back, exactly as MultigridGPUSubset:twoGrid does.
mg:metrics() returns relErr, count, frobErr of the last outer iteration (gpu.lua:173-200).
Extra table fields select the build's configurations: dim (2|3), real, smoother ('jacobi'|'rbgs'),
cycle ('V'|'F'), prolong ('pc'|'linear'), coarse_init ('fresh'|'warm'), coarse_bc
('zero'|'consistent'), device.  Defaults reproduce cpu.lua (2D, double, Jacobi 7+7, V-cycle,
injection, fresh zero coarse guess, ghost value 0).

Fields: mg.psi / mg.f return lua-matrix-style 1-based tables psi[i][j] (x = i) downloaded from
the GPU; mg.psiBuffer / mg.fBuffer return raw real* copies (cpu-raw.lua's .psi.buffer).
Errors from the library raise Lua errors (error()), as the reference's own failures do.

Not executable in this repository's CI (no Lua runtime in the image); the Python mirror in
../mgpoisson/solver.py is the tested twin of this file.
--]]
local ffi = require 'ffi'
local bit = require 'bit'

ffi.cdef[[
typedef struct mgp_ctx mgp_ctx;
typedef struct mgp_opts {
    int32_t struct_size;
    int32_t dim;
    int64_t n[3];
    int32_t real_bytes;
    int32_t nu1, nu2;
    int32_t smoother;
    int32_t cycle;
    int32_t prolong;
    int32_t coarse_init;
    int32_t coarse_bc;
    int32_t coarse_sweeps;
    int32_t err_mode;
    int32_t device;
    int32_t rank, world;
    int64_t gather_cells;
    uint8_t comm_id[128];
} mgp_opts;
int         mgp_version(void);
void        mgp_opts_default(mgp_opts* o);
int         mgp_create(mgp_ctx** out, const mgp_opts* o);
void        mgp_destroy(mgp_ctx* c);
const char* mgp_last_error(const mgp_ctx* c);
int         mgp_init_point_charge(mgp_ctx* c);
int         mgp_set_field(mgp_ctx* c, int level, int which, const void* src, int64_t count, int mem);
int         mgp_get_field(const mgp_ctx* c, int level, int which, void* dst, int64_t count, int mem);
int         mgp_cycle(mgp_ctx* c, double* err_out);
int         mgp_two_grid(mgp_ctx* c, double h, void* u, const void* f, int64_t L, int mem);
int         mgp_set_coarse_level(mgp_ctx* c, int64_t size);
typedef int (*mgp_coarse_fn)(void* user, double h, void* u, const void* f, int64_t size);
int         mgp_set_coarse_handoff(mgp_ctx* c, int64_t size, mgp_coarse_fn fn, void* user);
int         mgp_metrics(mgp_ctx* c, double* rel_err, int64_t* count, double* frob);
]]

local lib = ffi.load(os.getenv('MGP_LIBRARY') or 'mgpoisson')

local CODES = {
	smoother = {jacobi = 0, rbgs = 1},
	cycle = {V = 0, F = 1},
	prolong = {pc = 0, linear = 1},
	coarse_init = {fresh = 0, warm = 1},
	coarse_bc = {zero = 0, consistent = 1},
}

local function check(rc, ctx)
	if rc < 0 then error('libmgpoisson: ' .. ffi.string(lib.mgp_last_error(ctx)), 3) end
	return rc
end

local MultigridHIP = {}
MultigridHIP.__index = function(self, k)
	if k == 'psi' then return self:getMatrix(0) end
	if k == 'f' then return self:getMatrix(1) end
	if k == 'psiBuffer' then return self:getBuffer(0) end
	if k == 'fBuffer' then return self:getBuffer(1) end
	return rawget(MultigridHIP, k)
end

-- class defaults (cpu.lua:18-22, cpu-raw.lua:121-124)
MultigridHIP.debug = false
MultigridHIP.smooth = 7
MultigridHIP.epsilon = 1e-10
MultigridHIP.accuracy = 1e-10
MultigridHIP.maxiter = 1000

setmetatable(MultigridHIP, {
	__call = function(cls, ...)
		local self = setmetatable({}, cls)
		self:init(...)
		return self
	end,
})

function MultigridHIP:init(a, real, cpuDepth, engine)
	local args
	if type(a) == 'table' then
		args = a
		-- like cpu.lua:174-177: nil fields fall back to the class defaults
		rawset(self, 'maxiter', args.maxiter)
		rawset(self, 'epsilon', args.epsilon)
		rawset(self, 'errorCallback', args.errorCallback)
		if args.debug ~= nil then rawset(self, 'debug', args.debug) end
	else
		-- cpu-raw.lua positional protocol: persistent coarse buffers (cpu-raw.lua:221)
		args = {size = a, real = real, coarse_init = 'warm'}
		rawset(self, 'cpuDepth', cpuDepth)
	end
	local n = assert(tonumber(args.size), 'size is required')
	local dim = args.dim or 2
	rawset(self, 'real', args.real or 'double')
	rawset(self, 'dim', dim)
	rawset(self, 'size', n)
	local o = ffi.new('mgp_opts')
	lib.mgp_opts_default(o)
	o.dim = dim
	o.n[0], o.n[1], o.n[2] = n, n, (dim == 3 and n or 1)
	o.real_bytes = (self.real == 'float') and 4 or 8
	o.nu1, o.nu2 = args.smooth or self.smooth, args.smooth or self.smooth
	for field, map in pairs(CODES) do
		if args[field] ~= nil then o[field] = assert(map[args[field]], 'unknown ' .. field) end
	end
	if args.device then o.device = args.device end
	local pp = ffi.new('mgp_ctx*[1]')
	check(lib.mgp_create(pp, o), nil)
	rawset(self, 'ctx', ffi.gc(pp[0], lib.mgp_destroy))
	rawset(self, 'count', n * n * (dim == 3 and n or 1))
	rawset(self, 'ctype', (self.real == 'float') and 'float[?]' or 'double[?]')
	if cpuDepth then
		local L = bit.lshift(1, cpuDepth)
		if engine then
			-- cpu-gpu.lua:17-52: the callback runs engine:twoGrid on the level's host copies
			local cb = ffi.cast('mgp_coarse_fn', function(user, h, u, f, size)
				local ok = pcall(engine.twoGrid, engine, h, ffi.cast(self.ctype:gsub('%[%?%]', '*'), u),
					ffi.cast(self.ctype:gsub('%[%?%]', '*'), f), tonumber(size))
				return ok and 0 or 1
			end)
			rawset(self, 'handoff', cb)  -- keep the callback alive
			check(lib.mgp_set_coarse_handoff(self.ctx, L, cb, nil), self.ctx)
		else
			lib.mgp_set_coarse_level(self.ctx, L)  -- keeps the default switch when it does not fit
		end
	end
	check(lib.mgp_init_point_charge(self.ctx), self.ctx)  -- cpu.lua:180-193
end

function MultigridHIP:metrics()
	local rel, n, frob = ffi.new('double[1]'), ffi.new('int64_t[1]'), ffi.new('double[1]')
	check(lib.mgp_metrics(self.ctx, rel, n, frob), self.ctx)
	return rel[0], tonumber(n[0]), frob[0]
end

function MultigridHIP:getBuffer(which)
	local buf = ffi.new(self.ctype, self.count)
	check(lib.mgp_get_field(self.ctx, 0, which, buf, self.count, 0), self.ctx)
	return buf
end

-- 1-based nested table m[i][j] with i = x (cpu.lua's matrix indexing), 2D only
function MultigridHIP:getMatrix(which)
	local buf = self:getBuffer(which)
	local n = self.size
	if self.dim ~= 2 then return buf end
	local m = {}
	for i = 1, n do
		local row = {}
		for j = 1, n do row[j] = tonumber(buf[(i - 1) + n * (j - 1)]) end
		m[i] = row
	end
	return m
end

-- cpu.lua:196-206
function MultigridHIP:step()
	local err = ffi.new('double[1]')
	check(lib.mgp_cycle(self.ctx, err), self.ctx)
	if self.debug then print('err', err[0]) end
	return err[0]
end

-- cpu.lua:208-216, break rules included
function MultigridHIP:solve()
	if self.debug then print('#iter', 'err') end
	for iter = 1, self.maxiter do
		local err = self:step()
		if self.errorCallback and self.errorCallback(iter, err) then break end
		if err < self.epsilon or err ~= err or err == math.huge or err == -math.huge then break end
	end
end

-- cpu-raw.lua:239-258 / gpu.lua:348-373: two outer iterations
function MultigridHIP:run()
	print('#iter', 'err')
	for iter = 1, 2 do
		local err = self:step()
		print(iter, err)
		if err < self.accuracy or err ~= err then break end
	end
end

-- cpu-raw.lua:186 twoGrid(h, u, f, L) on raw host real* buffers (u updated in place)
function MultigridHIP:twoGrid(h, u, f, L)
	check(lib.mgp_two_grid(self.ctx, h, u, f, L, 0), self.ctx)
end

return MultigridHIP
