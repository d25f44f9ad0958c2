/// EngineCore/Native/Native.fs — the P/Invoke binding of libmafrix_rt.so (include/mafrix_rt.h)
/// and the GPU-backed IPixelIntegrator that Scene's constructor builds instead of
/// PixelIntegrator (Core/Integrator/Integrators.fs:143-172).
///
/// Compile position (fsharp/EngineCore.fsproj.diff): after Models\ObjModelLoader.fs, before
/// Scene\Scene.fs. Everything it opens is compiled earlier, and Scene.fs opens this module.
/// Checked against the reference's declarations by scripts/check_fsharp_shim.py
/// (tests/test_fsharp_shim.py); struct layouts follow mafrixraytracing_amd/abi.py, whose
/// offsets tests/test_abi.py checks against the C header.
module Engine.Core.Native

open System
open System.Runtime.InteropServices
open Engine.Core.Color
open Engine.Core.Point
open Engine.Core.Texture
open Engine.Core.Camera
open Engine.Core.Light
open Engine.Core.Material
open Engine.Core.Shapes.Triangle
open Engine.Core.Shapes.Rect
open Engine.Core.Shapes.Sphere
open Engine.Core.Interfaces.IHitable
open Engine.Core.Interfaces.ILight
open Engine.Core.Interfaces.ICamera
open Engine.Core.Interfaces.IMaterial
open Engine.Core.Interfaces.IIntegrator

// ---- blittable mirrors of the C structs (sequential layout, natural alignment) ----------------

/// mfx_prim (104 B): kind, material, p[4][3]
[<Struct; StructLayout(LayoutKind.Sequential)>]
type MfxPrim =
    val mutable kind : int32
    val mutable material : int32
    val mutable p0x : float
    val mutable p0y : float
    val mutable p0z : float
    val mutable p1x : float
    val mutable p1y : float
    val mutable p1z : float
    val mutable p2x : float
    val mutable p2y : float
    val mutable p2z : float
    val mutable p3x : float
    val mutable p3y : float
    val mutable p3z : float

/// mfx_quad_light (144 B): p[4][3], normal[3], intensity[3]
[<Struct; StructLayout(LayoutKind.Sequential)>]
type MfxQuadLight =
    val mutable p0x : float
    val mutable p0y : float
    val mutable p0z : float
    val mutable p1x : float
    val mutable p1y : float
    val mutable p1z : float
    val mutable p2x : float
    val mutable p2y : float
    val mutable p2z : float
    val mutable p3x : float
    val mutable p3y : float
    val mutable p3z : float
    val mutable nx : float
    val mutable ny : float
    val mutable nz : float
    val mutable ir : float
    val mutable ig : float
    val mutable ib : float

/// mfx_pinhole (144 B): position, direction, fov, aspect, topleft, right, down, derived, reserved
[<Struct; StructLayout(LayoutKind.Sequential)>]
type MfxPinhole =
    val mutable px : float
    val mutable py : float
    val mutable pz : float
    val mutable dx : float
    val mutable dy : float
    val mutable dz : float
    val mutable fov : float
    val mutable aspect : float
    val mutable tlx : float
    val mutable tly : float
    val mutable tlz : float
    val mutable rx : float
    val mutable ry : float
    val mutable rz : float
    val mutable dnx : float
    val mutable dny : float
    val mutable dnz : float
    val mutable derived : int32
    val mutable reserved : int32

/// mfx_scene_desc: prims, nprims, albedo, nmat, width, height, max_depth, light, camera
[<Struct; StructLayout(LayoutKind.Sequential)>]
type MfxSceneDesc =
    val mutable prims : nativeint
    val mutable nprims : int64
    val mutable albedo : nativeint
    val mutable nmat : int32
    val mutable width : int32
    val mutable height : int32
    val mutable maxDepth : int32
    val mutable light : MfxQuadLight
    val mutable camera : MfxPinhole

/// mfx_options (40 B): seed, device, flags, part_index, part_count, ndevices, render_ahead, devices
[<Struct; StructLayout(LayoutKind.Sequential)>]
type MfxOptions =
    val mutable seed : uint64
    val mutable device : int32
    val mutable flags : int32
    val mutable partIndex : int32
    val mutable partCount : int32
    val mutable ndevices : int32
    val mutable renderAhead : int32
    val mutable devices : nativeint

// ---- entry points --------------------------------------------------------------------------------

module Api =
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_create(MfxSceneDesc& scene, MfxOptions& opt, nativeint& ctx)
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern void mfx_destroy(nativeint ctx)
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_sample(nativeint ctx, int spp, nativeint frameXmajorRgba)
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_render_rgba8(nativeint ctx, int spp, byte[] rgbaYmajor)
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_reset(nativeint ctx)
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_stats(nativeint ctx, float& rays, float& seconds)
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern nativeint mfx_last_error()
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_device_count()
    [<DllImport("mafrix_rt", CallingConvention = CallingConvention.Cdecl)>]
    extern int mfx_abi_version()

/// include/mafrix_rt.h MFX_ABI_VERSION these declarations follow: a libmafrix_rt of another ABI
/// (struct layouts, call semantics) is refused at construction instead of failing silently.
let MFX_ABI_VERSION = 6
let MFX_F_NONE = 0
let MFX_F_HOST_BVH = 4      // build the traversal BVH on the CPU instead of the GPU (the same tree)
let DefaultSeed = 0x4D414652UL
/// Scene.Render's one-sample calls are served from batches of this many samples (mfx_options.render_ahead):
/// the batch is traced at once, the film add and post of all its calls run on the GPU ahead of them, and
/// the next batch is traced in the background while this one is served; every frame is the bytes of the
/// one-sample-per-call path. The library cuts it to what fits in a quarter of the free HBM.
let DefaultRenderAhead = 64

/// The library returns 0 or a negative MFX_E_* code; the reference signals failures by raising.
let check (rc : int) (what : string) =
    if rc <> 0 then
        failwithf "%s failed (%d): %s" what rc (Marshal.PtrToStringAnsi(Api.mfx_last_error()))

/// The loaded libmafrix_rt must be the ABI these declarations were written for.
let checkAbi () =
    let v = Api.mfx_abi_version()
    if v <> MFX_ABI_VERSION then
        failwithf "libmafrix_rt ABI %d, this binding needs ABI %d (rebuild or update the binding)" v MFX_ABI_VERSION

// ---- reference types -> ABI ----------------------------------------------------------------------

let private setP (m : byref<MfxPrim>, i : int, p : Point) =
    match i with
    | 0 -> m.p0x <- p.x; m.p0y <- p.y; m.p0z <- p.z
    | 1 -> m.p1x <- p.x; m.p1y <- p.y; m.p1z <- p.z
    | 2 -> m.p2x <- p.x; m.p2y <- p.y; m.p2z <- p.z
    | _ -> m.p3x <- p.x; m.p3y <- p.y; m.p3z <- p.z

/// state.shapes (boxed Triangle / Rect / Sphere structs, Scene.fs:168-177) -> mfx_prim[], in the
/// same order: it is the index space Bvh.Build sorts (BvhNode.fs:25).
let marshalShapes (shapes : IHitable[]) : MfxPrim[] =
    shapes |> Array.map (fun (s : IHitable) ->
        let mutable m = MfxPrim()
        match box s with
        | :? Triangle as t ->                       // Trangle.fs:98-119
            m.kind <- 0
            m.material <- t.material
            setP (&m, 0, t.v0)
            setP (&m, 1, t.v1)
            setP (&m, 2, t.v2)
        | :? Rect as r ->                           // Rect(v0,v1,v2,v3): trig1 = (v0,v1,v2), trig2 = (v0,v2,v3)
            m.kind <- 1
            m.material <- r.trig1.material
            setP (&m, 0, r.trig1.v0)
            setP (&m, 1, r.trig1.v1)
            setP (&m, 2, r.trig1.v2)
            setP (&m, 3, r.trig2.v2)
        | :? Sphere as sp ->                        // Sphere.fs:9-16
            m.kind <- 2
            m.material <- sp.material
            setP (&m, 0, sp.center)
            m.p1x <- sp.radius
        | _ -> failwith "Native: unsupported IHitable (Triangle, Rect and Sphere are the reference's)"
        m)

/// MaterialManager -> albedo table as LambertianBrdf sees it: Lambertian(a) and Metal(a, f) give
/// a (Material.fs:52, 68); SpecularTransmission's GetBxdf is LambertianBrdf(Color()) (:121).
let marshalAlbedo () : float[] =
    let mgr : MaterialManager = MaterialManager.GetManager()
    mgr.materials |> Array.collect (fun (mat : IMaterial) ->
        match mat with
        | :? SpecularTransmission -> [| 0.; 0.; 0. |]
        | _ ->
            let c : Color = mat.BaseColor()
            [| c.r; c.g; c.b |])

/// NewAreaLight (Light.fs:31-40) as Scene.fs:193 built it from a Rect.
let marshalLight (light : INewLight) : MfxQuadLight =
    match box light with
    | :? NewAreaLight as l ->
        let mutable q = MfxQuadLight()
        let v0 : Point = l.rect.trig1.v0
        let v1 : Point = l.rect.trig1.v1
        let v2 : Point = l.rect.trig1.v2
        let v3 : Point = l.rect.trig2.v2
        q.p0x <- v0.x; q.p0y <- v0.y; q.p0z <- v0.z
        q.p1x <- v1.x; q.p1y <- v1.y; q.p1z <- v1.z
        q.p2x <- v2.x; q.p2y <- v2.y; q.p2z <- v2.z
        q.p3x <- v3.x; q.p3y <- v3.y; q.p3z <- v3.z
        q.nx <- l.normal.x; q.ny <- l.normal.y; q.nz <- l.normal.z
        q.ir <- l.color.r; q.ig <- l.color.g; q.ib <- l.color.b
        q
    | _ -> failwith "Native: the light must be a NewAreaLight (Scene.fs:180-194)"

/// PinholeCamera after its constructor (Camera.fs:122-133), passed as derived fields
/// (derived = 1) so GetRay (Camera.fs:134-139) starts from identical bits.
let marshalCamera (camera : ICamera) : MfxPinhole =
    match box camera with
    | :? PinholeCamera as c ->
        let mutable p = MfxPinhole()
        p.px <- c.position.x; p.py <- c.position.y; p.pz <- c.position.z
        p.dx <- c.coord.forward.x; p.dy <- c.coord.forward.y; p.dz <- c.coord.forward.z
        p.fov <- c.fov
        p.aspect <- c.hori_size / c.vert_size
        p.tlx <- c.topleft.x; p.tly <- c.topleft.y; p.tlz <- c.topleft.z
        p.rx <- c.coord.right.x; p.ry <- c.coord.right.y; p.rz <- c.coord.right.z
        p.dnx <- c.coord.down.x; p.dny <- c.coord.down.y; p.dnz <- c.coord.down.z
        p.derived <- 1
        p
    | _ -> failwith "Native: the camera must be a PinholeCamera (Scene.fs:39-76)"

// ---- the GPU-backed pixel integrator ---------------------------------------------------------------

/// IPixelIntegrator (IIntegrator.fs:35-40) over one libmafrix_rt context.
///   devices = [||]: HIP device 0; devices = [|0..7|]: one context drives all eight GPUs of the
///   node by an image partition (GPU g traces one of each 8 consecutive 8-pixel tile rows of every frame and
///   batch, and copies its rows of each RGBA8 frame into the buffer): the frames are the one-GPU bytes.
/// Sample(n) writes the mean of n fresh samples per pixel straight into a pinned Color[w,h]
/// (Color is a sequential 4 x float struct, Color.fs:3-4; element (i,j) at i*h + j, as
/// mfx_sample writes it) and returns the Texture2D over it, as PixelIntegrator returns its own
/// texture (Integrators.fs:160-172).
type NativePixelIntegrator(shapes : IHitable[], light : INewLight, camera : ICamera,
                           width : int, height : int, devices : int[], seed : uint64) =
    let data : Color[,] = Array2D.zeroCreate<Color> width height
    let texture = Texture2D<Color>(data, width, height)
    let ctx =
        checkAbi ()
        let prims = marshalShapes shapes
        let albedo = marshalAlbedo ()
        let hp = GCHandle.Alloc(prims, GCHandleType.Pinned)
        let ha = GCHandle.Alloc(albedo, GCHandleType.Pinned)
        let hd = GCHandle.Alloc(devices, GCHandleType.Pinned)
        try
            let mutable d = MfxSceneDesc()
            d.prims <- hp.AddrOfPinnedObject()
            d.nprims <- int64 prims.Length
            d.albedo <- ha.AddrOfPinnedObject()
            d.nmat <- albedo.Length / 3
            d.width <- width
            d.height <- height
            d.maxDepth <- 3                                   // PathIntegrator(bvh, 3, light), Scene.fs:304
            d.light <- marshalLight light
            d.camera <- marshalCamera camera
            let mutable o = MfxOptions()
            o.seed <- seed
            o.device <- 0
            o.flags <- MFX_F_NONE
            o.partIndex <- 0
            o.partCount <- 1
            o.ndevices <- devices.Length
            o.renderAhead <- DefaultRenderAhead  // Scene.Render's one-sample calls served from batches of K samples
            o.devices <- (if devices.Length > 0 then hd.AddrOfPinnedObject() else 0n)
            let mutable c = 0n
            check (Api.mfx_create(&d, &o, &c)) "mfx_create"   // deep copy: the arrays are unpinned after
            c
        finally
            hp.Free()
            ha.Free()
            hd.Free()
    new(shapes : IHitable[], light : INewLight, camera : ICamera, width : int, height : int) =
        NativePixelIntegrator(shapes, light, camera, width, height, [||], DefaultSeed)
    member this.Handle = ctx
    /// Scene.Render on the GPU: Film.GetFrame(integrator, spp) + PostProcessAndToScreenBuffer
    /// (Film.fs:32-34, Scene.fs:315-333) into buffer = byte[w*h*4], y-major RGBA8.
    member this.RenderRgba8(spp : int, buffer : byte[]) =
        check (Api.mfx_render_rgba8(ctx, spp, buffer)) "mfx_render_rgba8"
    /// Film.Reset (Film.fs:26-30) of the GPU film.
    member this.Reset() = check (Api.mfx_reset ctx) "mfx_reset"
    /// Rays traced (primary + extension + shadow) and device seconds of the last call.
    member this.Stats() =
        let mutable rays = 0.
        let mutable seconds = 0.
        check (Api.mfx_stats(ctx, &rays, &seconds)) "mfx_stats"
        rays, seconds
    interface IPixelIntegrator with
        member this.Sample(n : int) =
            let h = GCHandle.Alloc(data, GCHandleType.Pinned)
            try
                check (Api.mfx_sample(ctx, n, h.AddrOfPinnedObject())) "mfx_sample"
            finally
                h.Free()
            texture
    interface IDisposable with
        member this.Dispose() = Api.mfx_destroy ctx
