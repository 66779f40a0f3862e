// TypeScript surface of the Node host (index.js): the reference's GpuContext / Renderer API
// (src/gpu_context.ts, src/renderer.ts) with WebGPU objects replaced by the HIP addon.
export declare const GS_ACCUM_FP32: 0;
export declare const GS_ACCUM_FP16_TARGET: 1;
export declare const GS_OUT_RGBA_F32: 0;
export declare const GS_OUT_RGBA_F16: 1;

export interface RenderOptions {
    accum?: number;          // GS_ACCUM_*
    outFormat?: number;      // GS_OUT_RGBA_*
    tMin?: number;           // early-stop transmittance (default 1e-4; 0 = never)
    stripIndex?: number;
    stripCount?: number;
    timing?: number;
    chunkFraction?: number;  // 0 = adaptive
    refQuirks?: number;      // 1: the reference's init-sort truncation (INTEGRATION.md section 5)
    listSplit?: number;      // 1: long tile lists in parallel segments (fp32-oracle bar, not bit-identical)
    deviceResident?: boolean;  // frames stay in HBM (renderDevice); Renderer.readback() copies one out
}

export declare class GpuContext {
    gpu: {api: 'hip'};
    adapter: {deviceIndex: number | number[]; deviceCount: number} | null;
    device: unknown | null;  // native gs_ctx handle
    constructor(gpu: {api: 'hip'}, adapter: {deviceIndex: number | number[]; deviceCount: number}, device: unknown);
    /** Rejects with a string when no HIP device exists (src/gpu_context.ts:12-26). */
    /** One HIP device, or a device group (row strips + one RCCL all-gather; image on the first). */
    static create(deviceIndex?: number | number[]): Promise<GpuContext>;
    destroy(): void;
}

export declare class PackedGaussians {
    gaussiansBuffer: ArrayBuffer;  // AoS records, src/ply.ts:249-257
    numGaussians: number;
    nShCoeffs: number;
    sphericalHarmonicsDegree: number;
    gaussianArrayLayout: {size: number};
    min_pos: number[];
    max_pos: number[];
    constructor(gaussiansBuffer: ArrayBuffer | ArrayBufferView, numGaussians: number, nShCoeffs?: number);
    /** The reference's `new PackedGaussians(plyArrayBuffer)` (src/ply.ts), parsed natively. */
    static fromPly(plyArrayBuffer: ArrayBuffer): PackedGaussians;
}

/** One entry of an INRIA cameras.json (src/camera.ts:7-16). */
export interface CameraRaw {
    id?: number;
    img_name?: string;
    width?: number;
    height?: number;
    position: number[];
    rotation: number[][];
    fx: number;
    fy: number;
}

export declare class Camera {
    height: number;
    width: number;
    viewMatrix: Float32Array;
    perspective: Float32Array;
    focalX: number;
    focalY: number;
    scaleModifier: number;
    constructor(height: number, width: number, viewMatrix: Float32Array, perspective: Float32Array,
                focalX: number, focalY: number, scaleModifier: number);
    static default(width: number, height: number): Camera;
    static fromJSON(rawCamera: CameraRaw, canvasW: number, canvasH: number): Camera;
    static lookAt(eye: number[], target: number[], width: number, height: number, fovy?: number,
                  near?: number, far?: number): Camera;
    getPosition(): Float32Array;
}

export interface InteractiveCameraLike {
    isDirty(): boolean;
    getCamera(): Camera;
}

export declare class HeadlessCamera implements InteractiveCameraLike {
    camera: Camera;
    dirty: boolean;
    constructor(camera: Camera);
    setNewCamera(camera: Camera): void;
    setDirty(): void;
    isDirty(): boolean;
    getCamera(): Camera;
}

export interface HeadlessCanvas {
    width: number;
    height: number;
    present?: boolean;                       // also produce the PostProcessRenderer image
    framebuffer?: Float32Array | Uint16Array;
    image?: Float32Array;
    onFrame?: (r: Renderer) => void;
    onError?: (e: Error) => void;
}

export declare class Renderer {
    canvas: HeadlessCanvas;
    interactiveCamera: InteractiveCameraLike;
    context: GpuContext;
    numGaussians: number;
    framebuffer: Float32Array | Uint16Array | null;  // SimpleRender.framebuffer contents (null when deviceResident)
    deviceFramebuffer: unknown;  // deviceResident: the framebuffer in HBM (addon handle)
    frames: number;
    static requestContext(gaussians: PackedGaussians, deviceIndex?: number | number[]): Promise<GpuContext>;
    constructor(canvas: HeadlessCanvas, interactiveCamera: InteractiveCameraLike, gaussians: PackedGaussians,
                context: GpuContext, fpsCounter?: {innerText: string; style: any}, options?: RenderOptions);
    /** Resolves after the next frame (src/renderer.ts:103-107). */
    destroy(): Promise<void>;
    resize(): void;
    /** deviceResident: the last frame copied to host memory once the frames in flight are done. */
    readback(target?: Float32Array | Uint16Array): Float32Array | Uint16Array;
    draw(nextFrameCallback: () => void): void;
    animate(forceDraw?: boolean): void;
    timings(): Record<string, number>;
}

export declare function addon(): any;
