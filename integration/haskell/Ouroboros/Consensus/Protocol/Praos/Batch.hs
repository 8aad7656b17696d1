{-# LANGUAGE DataKinds                #-}
{-# LANGUAGE ForeignFunctionInterface #-}
{-# LANGUAGE NamedFieldPuns           #-}
{-# LANGUAGE ScopedTypeVariables      #-}

-- | Batched Praos header validation on AMD MI355X GPUs (libpraos_hip.so).
--
-- The binding a maintainer adds beside
-- @ouroboros-consensus-protocol/src/ouroboros-consensus-protocol/Ouroboros/Consensus/Protocol/Praos.hs@.
-- It replaces, for the headers of one epoch at a time, the per-header crypto of
-- 'updateChainDepState' (Praos.hs:441-459: validateKESSignature :558-606 and
-- validateVRFSignature :528-556) and, for db-analyser's header revalidation
-- (Cardano/Tools/DBAnalyser/Analysis.hs:479-607, streaming loop :815-847), the whole
-- validateHeader fold (envelope + updateChainDepState) over stored header bytes.
--
-- GHC is not available where this repository is built, so this module is shipped as
-- source.  Its exact foreign-call sequence is exercised from C by
-- integration/c/ffi_harness.c (tests/test_gpu_ffi.py), and the struct layouts below
-- are checked against the C header by tests/test_abi.py (the "-- struct" lines).
--
-- Link: @extra-libraries: praos_hip@ (and @amdhip64@), include-dirs: include/.
module Ouroboros.Consensus.Protocol.Praos.Batch
  ( -- * Context (one GPU, or a group of several)
    PraosBatchCtx
  , withPraosBatchCtx
  , withPraosBatchDevices
  , praosBatchMembers
  , PraosBatchError (..)
  , praosSetPoolKeyStore
    -- * Per epoch
  , PraosParamsC (..)
  , praosSetEpoch
  , praosTickedEpochNonce
    -- * Headers from stored bytes
  , BatchResult (..)
  , praosValidateHeaderBytes
    -- * Headers from stored bytes, Storable vectors (Batch.Validate)
  , SpanResult (..)
  , ArenaPin (..)
  , praosValidateHeaderSpans
  , praosHostRegister
  , praosHostUnregister
  , praosSubmitHeaderBytes
  , praosDrainHeaderBytes
    -- * TPraos (Shelley..Alonzo) headers from stored bytes
  , TPraosBatchResult (..)
  , praosTickedEpochNonceTPraos
  , OverlayC (..)
  , praosSetOverlay
  , praosValidateTPraosHeaderBytes
  , praosValidateTPraosHeaderSpans
    -- * Whole ImmutableDB replay (db-analyser)
  , ReplayStats (..)
  , praosReplayImmutable
  , praosReplayImmutableTPraos
  , LedgerViewC (..)
  , praosReplayImmutableViews
    -- * ImmutableDB chunk validation (verifyBlockIntegrity batched)
  , ChunkValidation (..)
  , verifyChunkIntegrity
  , praosVerifyBlockIntegrity
    -- * Error reconstruction (typed constructors: module Batch.Errors)
  , verdictToError
  ) where

import           Control.Exception (Exception, bracket, bracket_, throwIO)
import           Control.Monad (forM_, when)
import qualified Data.ByteString as BS
import qualified Data.ByteString.Unsafe as BSU
import qualified Data.Vector.Storable as VS
import qualified Data.Vector.Storable.Mutable as VSM
import           Data.Ratio (denominator, numerator)
import           Data.Word (Word16, Word32, Word64, Word8)
import           Foreign
import           Foreign.C.String (CString, peekCString, withCString)
import           Foreign.C.Types (CInt (..), CSize (..))

-- ---------------------------------------------------------------- C ABI (include/praos_hip.h)

data PraosCtx
data PraosGroup

-- struct praos_params (40 bytes): slots_per_kes_period@0 max_kes_evo@8 f_is_one@16 vrf_check_output@20 c_raw@24
-- struct praos_pool (76 bytes): hash28@0 vrf_hash32@28 sigma_fp@60
-- struct praos_headers (120 bytes): n@0 slot@8 cold_vk@16 ocert_n@56 body_bytes_len@112
-- struct praos_header_bytes (40 bytes): n@0 bytes@8 bytes_len@16 off@24 len@32
-- struct praos_out (40 bytes): bits@0 pool_idx@8 beta@16 leader@24 nonce@32
-- struct praos_nonce (36 bytes): hash@0 neutral@32
-- struct praos_chain_state (232 bytes): last_slot_origin@0 last_slot@8 counter_hash28@16 counter@24 m@32 cap@40 evolving@48 candidate@84 epoch_nonce@120 lab@156 last_epoch_block@192
-- struct praos_epoch_info (32 bytes): epoch_base_slot@0 epoch_base_no@8 epoch_length@16 stability_window@24
-- struct praos_envelope (120 bytes): block_no@0 header_hash@8 header_size@16 body_size@24 tip_is_origin@32 tip_slot@40 tip_block_no@48 tip_hash@56 max_major_pv@88 lv_prot_major@96 max_header_size@104 max_body_size@112
-- struct praos_replay_stats (80 bytes): skipped@0 headers@8 validated@16 stop_index@24 stop_verdict@32 epochs@36 batches@40 chunks@44 ms_io@48 ms_device@56 ms_fold@64 ms_nonce@72
-- struct praos_decoded (168 bytes): status@0 block_no@8 slot@16 prev_hash@24 prev_is_genesis@32 cold_vk@40 body_size@72 ocert_n@96 header_hash@160
-- struct praos_tpraos_headers (136 bytes): h@0 leader_out@120 leader_proof@128
-- struct praos_tpraos_out (40 bytes): bits@0 pool_idx@8 beta_eta@16 beta_leader@24 nonce@32
-- struct praos_ledger_view (48 bytes): first_epoch@0 pools@8 npools@16 reserved@20 lv_prot_major@24 max_header_size@32 max_body_size@40

foreign import ccall safe "praos_open"        c_open        :: CInt -> IO (Ptr PraosCtx)
foreign import ccall safe "praos_close"       c_close       :: Ptr PraosCtx -> IO ()
foreign import ccall safe "praos_last_error"  c_last_error  :: Ptr PraosCtx -> IO CString
foreign import ccall safe "praos_abi_version" c_abi_version :: IO CInt
foreign import ccall safe "praos_set_option"  c_set_option  :: Ptr PraosCtx -> CInt -> CInt -> IO CInt
foreign import ccall safe "praos_set_epoch"   c_set_epoch
  :: Ptr PraosCtx -> Ptr Word8 -> Ptr () -> Word32 -> Ptr () -> IO CInt
foreign import ccall safe "praos_ticked_epoch_nonce" c_ticked_epoch_nonce
  :: Ptr () -> Ptr () -> Word64 -> Ptr () -> IO CInt
foreign import ccall safe "praos_verify_header_bytes" c_verify_header_bytes
  :: Ptr PraosCtx -> Ptr () -> Ptr () -> Ptr () -> IO CInt
foreign import ccall safe "praos_validate_headers" c_validate_headers
  :: Ptr PraosCtx -> Ptr () -> Ptr Word8 -> Ptr Word8 -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> Ptr Word8 -> Ptr CSize -> Ptr CSize -> IO CInt
foreign import ccall safe "praos_host_register" c_host_register
  :: Ptr PraosCtx -> Ptr Word8 -> CSize -> IO CInt
foreign import ccall safe "praos_host_unregister" c_host_unregister
  :: Ptr PraosCtx -> Ptr Word8 -> IO CInt
foreign import ccall safe "praos_state_encode" c_state_encode
  :: Ptr () -> Ptr Word8 -> CSize -> Ptr CSize -> IO CInt
foreign import ccall safe "praos_state_decode" c_state_decode
  :: Ptr Word8 -> CSize -> Ptr () -> IO CInt
foreign import ccall safe "praos_replay_immutable" c_replay_immutable
  :: Ptr PraosCtx -> CString -> Ptr () -> Word32 -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> CSize -> Ptr Word8 -> CSize -> Ptr () -> IO CInt
-- TPraos (include/praos_hip.h: praos_tpraos_*)
foreign import ccall safe "praos_tpraos_ticked_epoch_nonce" c_tpraos_ticked_epoch_nonce
  :: Ptr () -> Ptr () -> Word64 -> Ptr () -> Ptr () -> IO CInt
foreign import ccall safe "praos_verify_tpraos_header_bytes" c_verify_tpraos_header_bytes
  :: Ptr PraosCtx -> Ptr () -> Ptr () -> Ptr () -> Ptr Word8 -> Ptr Word8 -> IO CInt
foreign import ccall safe "praos_tpraos_update_chain_dep_state" c_tpraos_update_chain_dep_state
  :: Ptr PraosCtx -> Ptr () -> Ptr Word8 -> Ptr Word8 -> Ptr () -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> Ptr Word8 -> Ptr Word16 -> Ptr CSize -> Ptr CSize -> IO CInt
foreign import ccall safe "praos_set_overlay" c_set_overlay :: Ptr PraosCtx -> Ptr () -> IO CInt
foreign import ccall safe "praos_group_set_overlay" c_group_set_overlay :: Ptr PraosGroup -> Ptr () -> IO CInt
foreign import ccall safe "praos_replay_immutable_tpraos" c_replay_immutable_tpraos
  :: Ptr PraosCtx -> CString -> Ptr () -> Word32 -> Ptr () -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> CSize -> Ptr Word8 -> Ptr Word16 -> CSize -> Ptr () -> IO CInt
-- several GPUs (include/praos_hip.h: praos_group_*): shards of one batch, or consecutive
-- replay batches, on the members; outputs in place; the fold on member 0
foreign import ccall safe "praos_group_open"  c_group_open  :: Ptr CInt -> CInt -> IO (Ptr PraosGroup)
foreign import ccall safe "praos_group_close" c_group_close :: Ptr PraosGroup -> IO ()
foreign import ccall safe "praos_group_size"  c_group_size  :: Ptr PraosGroup -> IO CInt
foreign import ccall safe "praos_group_ctx"   c_group_ctx   :: Ptr PraosGroup -> CInt -> IO (Ptr PraosCtx)
foreign import ccall safe "praos_group_last_error" c_group_last_error :: Ptr PraosGroup -> IO CString
foreign import ccall safe "praos_group_set_option" c_group_set_option :: Ptr PraosGroup -> CInt -> CInt -> IO CInt
foreign import ccall safe "praos_group_set_epoch" c_group_set_epoch
  :: Ptr PraosGroup -> Ptr Word8 -> Ptr () -> Word32 -> Ptr () -> IO CInt
foreign import ccall safe "praos_group_verify_header_bytes" c_group_verify_header_bytes
  :: Ptr PraosGroup -> Ptr () -> Ptr () -> Ptr () -> IO CInt
foreign import ccall safe "praos_group_verify_tpraos_header_bytes" c_group_verify_tpraos_header_bytes
  :: Ptr PraosGroup -> Ptr () -> Ptr () -> Ptr () -> Ptr Word8 -> Ptr Word8 -> IO CInt
foreign import ccall safe "praos_group_host_register" c_group_host_register
  :: Ptr PraosGroup -> Ptr Word8 -> CSize -> IO CInt
foreign import ccall safe "praos_group_host_unregister" c_group_host_unregister
  :: Ptr PraosGroup -> Ptr Word8 -> IO CInt
foreign import ccall safe "praos_group_replay_immutable" c_group_replay_immutable
  :: Ptr PraosGroup -> CString -> Ptr () -> Word32 -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> CSize -> Ptr Word8 -> CSize -> Ptr () -> IO CInt
foreign import ccall safe "praos_group_replay_immutable_tpraos" c_group_replay_immutable_tpraos
  :: Ptr PraosGroup -> CString -> Ptr () -> Word32 -> Ptr () -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> CSize -> Ptr Word8 -> Ptr Word16 -> CSize -> Ptr () -> IO CInt
-- ABI 14: a ledger view per epoch in the replay; block integrity (ImmutableDB chunk validation)
foreign import ccall safe "praos_replay_immutable_views" c_replay_immutable_views
  :: Ptr PraosCtx -> CString -> Ptr () -> Word32 -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> CSize -> Ptr Word8 -> CSize -> Ptr () -> IO CInt
foreign import ccall safe "praos_group_replay_immutable_views" c_group_replay_immutable_views
  :: Ptr PraosGroup -> CString -> Ptr () -> Word32 -> Ptr () -> Ptr () -> Ptr () -> Ptr ()
  -> CSize -> Ptr Word8 -> CSize -> Ptr () -> IO CInt
foreign import ccall safe "praos_verify_block_integrity" c_verify_block_integrity
  :: Ptr PraosCtx -> Ptr () -> Word64 -> Ptr Word8 -> Ptr Word8 -> IO CInt
foreign import ccall safe "praos_group_verify_block_integrity" c_group_verify_block_integrity
  :: Ptr PraosGroup -> Ptr () -> Word64 -> Ptr Word8 -> Ptr Word8 -> IO CInt

-- ABI 15: the streaming form of praos_verify_header_bytes (three calls in flight per context)
foreign import ccall safe "praos_verify_header_bytes_submit" c_verify_header_bytes_submit
  :: Ptr PraosCtx -> Ptr () -> Ptr () -> Ptr () -> IO CInt
foreign import ccall safe "praos_verify_drain" c_verify_drain :: Ptr PraosCtx -> IO CInt

abiVersion :: CInt
abiVersion = 15

-- ---------------------------------------------------------------- context

-- | One GPU (a praos_ctx), or a group of several (a praos_group: one context per device,
-- batches split into contiguous shards, replay batches dealt to the members in turn) together
-- with its member 0, on which the sequential fold runs.  Every entry point below takes either.
data PraosBatchCtx
  = PraosBatchCtx !(Ptr PraosCtx)
  | PraosBatchGroup !(Ptr PraosGroup) !(Ptr PraosCtx) !Int

data PraosBatchError = PraosBatchError !Int !String
  deriving Show
instance Exception PraosBatchError

-- | One context per GPU (device ordinal) and per Haskell thread that uses it; calls block
-- (the foreign imports are @safe@, so other Haskell threads keep running).
withPraosBatchCtx :: Int -> (PraosBatchCtx -> IO a) -> IO a
withPraosBatchCtx dev k = do
  v <- c_abi_version
  when (v /= abiVersion) $ throwIO (PraosBatchError (-2) ("libpraos_hip ABI " ++ show v))
  bracket (c_open (fromIntegral dev)) c_close $ \p -> do
    when (p == nullPtr) $ throwIO (PraosBatchError (-1) ("praos_open " ++ show dev))
    k (PraosBatchCtx p)

-- | The GPUs of one node as one batch context (SURVEY sec. 8e: an epoch's headers shard by
-- contiguous slot range, no exchange between devices).  One device is 'withPraosBatchCtx';
-- several are a praos_group (a device may repeat: several contexts on one GPU).
withPraosBatchDevices :: [Int] -> (PraosBatchCtx -> IO a) -> IO a
withPraosBatchDevices [] _ = throwIO (PraosBatchError (-1) "withPraosBatchDevices: no device")
withPraosBatchDevices [dev] k = withPraosBatchCtx dev k
withPraosBatchDevices devs k = do
  v <- c_abi_version
  when (v /= abiVersion) $ throwIO (PraosBatchError (-2) ("libpraos_hip ABI " ++ show v))
  let m = length devs
  bracket (withArray (map fromIntegral devs) $ \dp -> c_group_open dp (fromIntegral m)) c_group_close $ \g -> do
    when (g == nullPtr) $ throwIO (PraosBatchError (-1) ("praos_group_open " ++ show devs))
    c0 <- c_group_ctx g 0
    k (PraosBatchGroup g c0 m)

-- | Devices (contexts) a batch context spreads over.
praosBatchMembers :: PraosBatchCtx -> Int
praosBatchMembers (PraosBatchCtx _) = 1
praosBatchMembers (PraosBatchGroup _ _ m) = m

-- | The context the fold and the codecs run on (member 0 of a group).
ctxPtr :: PraosBatchCtx -> Ptr PraosCtx
ctxPtr (PraosBatchCtx p) = p
ctxPtr (PraosBatchGroup _ p _) = p

-- | PRAOS_OPT_POOL_KEYS (7): keep the cold-key and VRF-key cache entries across calls on
-- this context (a node validating batch after batch of one epoch sees the same pool keys);
-- verdicts are identical either way.  On by default inside the replay entry points.
praosSetPoolKeyStore :: PraosBatchCtx -> Bool -> IO ()
praosSetPoolKeyStore ctx on = check ctx $ case ctx of
  PraosBatchCtx p -> c_set_option p 7 (if on then 1 else 0)
  PraosBatchGroup g _ _ -> c_group_set_option g 7 (if on then 1 else 0)

-- | A batch call's return code: the group's error text for group calls, the context's otherwise.
check :: PraosBatchCtx -> IO CInt -> IO ()
check ctx act = do
  rc <- act
  when (rc /= 0) $ do
    msg <- case ctx of
      PraosBatchCtx p -> c_last_error p >>= peekCString
      PraosBatchGroup g _ _ -> c_group_last_error g >>= peekCString
    throwIO (PraosBatchError (fromIntegral rc) msg)

-- | A call on one context (the fold on member 0 of a group).
checkCtx :: Ptr PraosCtx -> IO CInt -> IO ()
checkCtx p = check (PraosBatchCtx p)

-- | praos_verify_header_bytes, or its group form (shards on the members, outputs in place).
verifyHeaderBytes :: PraosBatchCtx -> Ptr () -> Ptr () -> Ptr () -> IO ()
verifyHeaderBytes ctx hb out dec = check ctx $ case ctx of
  PraosBatchCtx p -> c_verify_header_bytes p hb out dec
  PraosBatchGroup g _ _ -> c_group_verify_header_bytes g hb out dec

-- | The streaming form of 'verifyHeaderBytes' (praos_verify_header_bytes_submit): the call is
-- queued and returns; its outputs are written by the third submit after it (a context keeps
-- three calls in flight, the next ones' uploads and stage V under this one's key chains) or by
-- 'praosDrainHeaderBytes'.  The header-bytes struct, the arena and the output arrays must stay
-- alive and unchanged until then.  A group runs the blocking call.
praosSubmitHeaderBytes :: PraosBatchCtx -> Ptr () -> Ptr () -> Ptr () -> IO ()
praosSubmitHeaderBytes ctx hb out dec = check ctx $ case ctx of
  PraosBatchCtx p -> c_verify_header_bytes_submit p hb out dec
  PraosBatchGroup g _ _ -> c_group_verify_header_bytes g hb out dec

-- | Every submitted call's outputs written (praos_verify_drain).
praosDrainHeaderBytes :: PraosBatchCtx -> IO ()
praosDrainHeaderBytes ctx = case ctx of
  PraosBatchCtx p -> check ctx (c_verify_drain p)
  PraosBatchGroup {} -> pure ()

verifyTPraosHeaderBytes :: PraosBatchCtx -> Ptr () -> Ptr () -> Ptr () -> IO ()
verifyTPraosHeaderBytes ctx hb out dec = check ctx $ case ctx of
  PraosBatchCtx p -> c_verify_tpraos_header_bytes p hb out dec nullPtr nullPtr
  PraosBatchGroup g _ _ -> c_group_verify_tpraos_header_bytes g hb out dec nullPtr nullPtr

-- | Who page-locks a batch's arena: 'PinForCall' -- the call registers it for its own
-- duration when it is 64 MiB or more -- or 'PinnedByCaller': the caller registered it once
-- ('praosHostRegister', e.g. an arena reused epoch after epoch and re-registered only when it
-- grows), so the call's time holds no pinning.
data ArenaPin = PinForCall | PinnedByCaller
  deriving (Eq, Show)

-- | praos_host_register (every member of a group): uploads from inside the range go by direct
-- DMA.  Pair with 'praosHostUnregister' before the buffer is freed or moved.
praosHostRegister :: PraosBatchCtx -> Ptr Word8 -> Int -> IO ()
praosHostRegister ctx ap alen = check ctx $ case ctx of
  PraosBatchCtx p -> c_host_register p ap (fromIntegral alen)
  PraosBatchGroup g _ _ -> c_group_host_register g ap (fromIntegral alen)

praosHostUnregister :: PraosBatchCtx -> Ptr Word8 -> IO ()
praosHostUnregister ctx ap = check ctx $ case ctx of
  PraosBatchCtx p -> c_host_unregister p ap
  PraosBatchGroup g _ _ -> c_group_host_unregister g ap

-- | The arena page-locked for the duration of the action when it is 64 MiB or more
-- (praos_host_register: the upload goes by direct DMA, no staging copy; a group pins it
-- once for every member) and the caller has not pinned it.  The unregister runs whatever the
-- action throws (a failing batch call), so a GHC-owned buffer is never freed while still
-- page-locked.
withRegisteredArena :: PraosBatchCtx -> ArenaPin -> Ptr Word8 -> Int -> IO a -> IO a
withRegisteredArena ctx pin ap alen act
  | pin == PinnedByCaller || alen < 64 * 1024 * 1024 = act
  | otherwise = bracket_ (praosHostRegister ctx ap alen) (praosHostUnregister ctx ap) act

-- ---------------------------------------------------------------- marshalling helpers

-- | Little-endian bytes of a non-negative Integer (Fixed E34 raw values, int128 two's
-- complement for activeSlotLog).
pokeLE :: Ptr Word8 -> Int -> Integer -> IO ()
pokeLE p n x = forM_ [0 .. n - 1] $ \i ->
  pokeByteOff p i (fromIntegral ((x `mod` 2 ^ (128 :: Int)) `shiftR` (8 * i)) :: Word8)

pokeBS :: Ptr a -> Int -> BS.ByteString -> IO ()
pokeBS p off bs = BSU.unsafeUseAsCStringLen bs $ \(src, n) -> copyBytes (p `plusPtr` off) (castPtr src) n

-- | PraosParams as the ABI wants them (praos_params): slotsPerKESPeriod, maxKESEvo,
-- f == 1, activeSlotLog f (unActiveSlotLog, Fixed E34 raw, <= 0), and whether
-- 'VRF.verifyCertified' compares the certified output with the proof's hash.
--
-- ppVrfCheckOutput: cardano-crypto-class >= 2.1 (the CHaP index-state this snapshot
-- pins, cabal.project:15-20) defines @verifyCertified ctx vk a c = verifyVRF ctx vk a
-- (certifiedProof c) == Just (certifiedOutput c)@ -- True, the default a caller should pass.
-- Older cardano-crypto-class releases (1.x: @verifyVRF ... (output, proof) -> Bool@ whose
-- PraosVRF instance ignored the output) correspond to False.  Either way the batch reports
-- both facts: PRAOS_BIT_VRF_PROOF (proof) and PRAOS_BIT_VRF_OUTPUT (output mismatch, set
-- only when checked).
data PraosParamsC = PraosParamsC
  { ppSlotsPerKESPeriod :: !Word64
  , ppMaxKESEvo         :: !Word64
  , ppFIsOne            :: !Bool
  , ppActiveSlotLogRaw  :: !Integer
  , ppVrfCheckOutput    :: !Bool
  }

withParams :: PraosParamsC -> (Ptr () -> IO a) -> IO a
withParams pp k = allocaBytes 40 $ \p -> do
  fillBytes p 0 40
  pokeByteOff p 0 (ppSlotsPerKESPeriod pp)
  pokeByteOff p 8 (ppMaxKESEvo pp)
  pokeByteOff p 16 (if ppFIsOne pp then 1 else 0 :: Word32)
  pokeByteOff p 20 (if ppVrfCheckOutput pp then 1 else 0 :: Word32)
  pokeLE (p `plusPtr` 24) 16 (ppActiveSlotLogRaw pp)
  k (castPtr p)

-- | PoolDistr entries: (KeyHash 'StakePool bytes, VRF key hash bytes, sigma as
-- Fixed E34 raw = floor (sigma * 10^34), i.e. fromRational individualPoolStake).
withPools :: [(BS.ByteString, BS.ByteString, Integer)] -> (Ptr () -> Word32 -> IO a) -> IO a
withPools pools k = allocaBytes (76 * max 1 (length pools)) $ \p -> do
  forM_ (zip [0 ..] pools) $ \(i, (hk, vrf, sigma)) -> do
    let q = p `plusPtr` (76 * i)
    pokeBS q 0 hk
    pokeBS q 28 vrf
    pokeLE (q `plusPtr` 60) 16 sigma
  k (castPtr p) (fromIntegral (length pools))

-- | A nonce: Nothing = NeutralNonce.
pokeNonce :: Ptr a -> Int -> Maybe BS.ByteString -> IO ()
pokeNonce p off mn = case mn of
  Nothing -> fillBytes (p `plusPtr` off) 0 32 >> pokeByteOff p (off + 32) (1 :: Word32)
  Just h  -> pokeBS p off h >> pokeByteOff p (off + 32) (0 :: Word32)

peekNonce :: Ptr a -> Int -> IO (Maybe BS.ByteString)
peekNonce p off = do
  neutral :: Word32 <- peekByteOff p (off + 32)
  if neutral /= 0 then pure Nothing else Just <$> BS.packCStringLen (castPtr (p `plusPtr` off), 32)

-- ---------------------------------------------------------------- per epoch

-- | praos_set_epoch: the epoch nonce (tickChainDepState's, see 'praosTickedEpochNonce'),
-- the PoolDistr of the ledger view and the protocol parameters.
praosSetEpoch :: PraosBatchCtx -> Maybe BS.ByteString -> [(BS.ByteString, BS.ByteString, Integer)]
              -> PraosParamsC -> IO ()
praosSetEpoch ctx eta0 pools pp =
  withPools pools $ \pp' np -> withParams pp $ \par ->
    case eta0 of
      Nothing -> set nullPtr pp' np par
      Just e  -> BSU.unsafeUseAsCString e $ \ep -> set (castPtr ep) pp' np par
  where
    set ep pp' np par = check ctx $ case ctx of
      PraosBatchCtx p -> c_set_epoch p ep pp' np par
      PraosBatchGroup g _ _ -> c_group_set_epoch g ep pp' np par

-- | The serialised PraosState (Praos.hs:274-310) the fold reads and writes; the ABI
-- takes the same CBOR through praos_state_encode / praos_state_decode, so the Haskell
-- side keeps its own PraosState and converts at batch boundaries.
withChainState :: BS.ByteString -> Int -> (Ptr () -> IO a) -> IO a
withChainState cbor cap k =
  allocaBytes 232 $ \st -> allocaBytes (28 * cap) $ \hk -> allocaBytes (8 * cap) $ \ctr -> do
    fillBytes st 0 232
    pokeByteOff st 16 hk
    pokeByteOff st 24 ctr
    pokeByteOff st 40 (fromIntegral cap :: CSize)
    BSU.unsafeUseAsCStringLen cbor $ \(src, n) -> do
      rc <- c_state_decode (castPtr src) (fromIntegral n) (castPtr st)
      when (rc /= 0) $ throwIO (PraosBatchError (fromIntegral rc) "praos_state_decode")
    k (castPtr st)

encodeChainState :: Ptr () -> IO BS.ByteString
encodeChainState st = alloca $ \lenp -> do
  _ <- c_state_encode st nullPtr 0 lenp
  n <- peek lenp
  allocaBytes (fromIntegral n) $ \buf -> do
    rc <- c_state_encode st buf n lenp
    when (rc /= 0) $ throwIO (PraosBatchError (fromIntegral rc) "praos_state_encode")
    BS.packCStringLen (castPtr buf, fromIntegral n)

withEpochInfo :: (Word64, Word64, Word64, Word64) -> (Ptr () -> IO a) -> IO a
withEpochInfo (baseSlot, baseNo, len, window) k = allocaBytes 32 $ \p -> do
  pokeByteOff p 0 baseSlot >> pokeByteOff p 8 baseNo >> pokeByteOff p 16 len >> pokeByteOff p 24 window
  k (castPtr p)

-- | tickChainDepState's epoch nonce at a slot (praos_ticked_epoch_nonce).
praosTickedEpochNonce :: BS.ByteString -> (Word64, Word64, Word64, Word64) -> Word64 -> IO (Maybe BS.ByteString)
praosTickedEpochNonce stateCbor ei slot =
  withChainState stateCbor (1 + 65536) $ \st -> withEpochInfo ei $ \eip -> allocaBytes 36 $ \out -> do
    rc <- c_ticked_epoch_nonce st eip slot (castPtr out)
    when (rc /= 0) $ throwIO (PraosBatchError (fromIntegral rc) "praos_ticked_epoch_nonce")
    peekNonce out 0

-- ---------------------------------------------------------------- headers from stored bytes

-- | One epoch's stored headers validated (validateHeader over the batch): per-header
-- verdicts (PRAOS_V_*), check bits, the chain stop and the state / tip after it.
data BatchResult = BatchResult
  { brVerdicts  :: ![Word8]
  , brBits      :: ![Word16]
  , brChainStop :: !Int
  , brState     :: !BS.ByteString          -- PraosState CBOR after the last valid header
  , brTip       :: !(Maybe (Word64, Word64, BS.ByteString))
  }

-- | Envelope limits of the ledger view: (praosMaxMajorPV, pvMajor lvProtocolVersion,
-- lvMaxHeaderSize, lvMaxBodySize).
type EnvLimits = (Word64, Word64, Word64, Word64)

-- | praos_verify_header_bytes (decode + all crypto on the GPU) then praos_validate_headers
-- (envelope, updateChainDepState) for the stored headers of one epoch, in chain order.
-- The epoch must have been installed with 'praosSetEpoch'.
praosValidateHeaderBytes :: PraosBatchCtx -> (Word64, Word64, Word64, Word64) -> EnvLimits
                         -> Maybe (Word64, Word64, BS.ByteString) -> BS.ByteString -> [BS.ByteString]
                         -> IO BatchResult
praosValidateHeaderBytes ctx ei (maxPV, pvMajor, maxHS, maxBS) tip stateCbor hdrs = do
  let n = length hdrs
      arena = BS.concat hdrs
      lens = map BS.length hdrs
      offs = take n (scanl (+) 0 lens)
  BSU.unsafeUseAsCString arena $ \ap ->
    withArray (map fromIntegral offs :: [Word64]) $ \offp ->
    withArray (map fromIntegral lens :: [Word32]) $ \lenp ->
    allocaBytes 40 $ \hb ->
    allocaArray n $ \(bits :: Ptr Word16) -> allocaArray n $ \(pidx :: Ptr Int32) ->
    allocaBytes (32 * n) $ \nonce ->
    allocaArray n $ \(slot :: Ptr Word64) -> allocaArray n $ \(bno :: Ptr Word64) ->
    allocaArray n $ \(ocn :: Ptr Word64) -> allocaArray n $ \(bsz :: Ptr Word32) ->
    allocaBytes (32 * n) $ \prev -> allocaBytes n $ \gen -> allocaBytes (32 * n) $ \cold ->
    allocaBytes (32 * n) $ \hh -> allocaBytes 168 $ \dec -> allocaBytes 40 $ \out ->
    allocaBytes 120 $ \hv -> allocaBytes 120 $ \env -> allocaArray n $ \(verdict :: Ptr Word8) ->
    alloca $ \stopp -> alloca $ \donep ->
    withChainState stateCbor (n + 65536) $ \st -> withEpochInfo ei $ \eip -> do
      pokeByteOff hb 0 (fromIntegral n :: CSize) >> pokeByteOff hb 8 ap
      pokeByteOff hb 16 (fromIntegral (BS.length arena) :: CSize)
      pokeByteOff hb 24 offp >> pokeByteOff hb 32 lenp
      fillBytes out 0 40 >> pokeByteOff out 0 bits >> pokeByteOff out 8 pidx >> pokeByteOff out 32 nonce
      fillBytes dec 0 168
      pokeByteOff dec 8 bno >> pokeByteOff dec 16 slot >> pokeByteOff dec 24 prev >> pokeByteOff dec 32 gen
      pokeByteOff dec 40 cold >> pokeByteOff dec 72 bsz >> pokeByteOff dec 96 ocn >> pokeByteOff dec 160 hh
      verifyHeaderBytes ctx (castPtr hb) (castPtr out) (castPtr dec)
      -- praos_headers: n, slot, cold_vk, ocert_n are what the fold reads
      fillBytes hv 0 120
      pokeByteOff hv 0 (fromIntegral n :: CSize) >> pokeByteOff hv 8 slot >> pokeByteOff hv 16 cold
      pokeByteOff hv 56 ocn
      fillBytes env 0 120
      pokeByteOff env 0 bno >> pokeByteOff env 8 hh >> pokeByteOff env 16 lenp >> pokeByteOff env 24 bsz
      case tip of
        Nothing -> pokeByteOff env 32 (1 :: Int32)
        Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
      pokeByteOff env 88 maxPV >> pokeByteOff env 96 pvMajor >> pokeByteOff env 104 maxHS
      pokeByteOff env 112 maxBS
      checkCtx (ctxPtr ctx) (c_validate_headers (ctxPtr ctx) (castPtr hv) prev gen (castPtr out) (castPtr env) eip st
                                                verdict stopp donep)
      stop <- peek stopp
      vs <- peekArray n verdict
      bs <- peekArray n bits
      st' <- encodeChainState st
      origin :: Int32 <- peekByteOff env 32
      tip' <- if origin /= 0 then pure Nothing else do
        s <- peekByteOff env 40
        b <- peekByteOff env 48
        h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
        pure (Just (s, b, h))
      pure (BatchResult vs bs (fromIntegral stop) st' tip')

-- | 'praosValidateHeaderSpans'' result: the chain stop, the PraosState CBOR and the tip
-- after the last valid header.
data SpanResult = SpanResult
  { srChainStop :: !Int
  , srState     :: !BS.ByteString
  , srTip       :: !(Maybe (Word64, Word64, BS.ByteString))
  }

-- | 'praosValidateHeaderBytes' over Storable vectors: the stored header spans in one arena
-- with their offsets and lengths, the verdicts (PRAOS_V_*) and check bits (PRAOS_BIT_*)
-- written into the caller's mutable vectors (length n each).  An arena of 64 MiB or more is
-- page-locked for the call (praos_host_register: the upload goes by direct DMA, no staging
-- copy).  The decoded fields and nonce values the fold reads stay in one allocation of 157
-- bytes per header.
praosValidateHeaderSpans :: PraosBatchCtx -> (Word64, Word64, Word64, Word64) -> EnvLimits
                         -> Maybe (Word64, Word64, BS.ByteString) -> BS.ByteString -> ArenaPin -> BS.ByteString
                         -> VS.Vector Word64 -> VS.Vector Word32 -> VSM.IOVector Word8 -> VSM.IOVector Word16
                         -> IO SpanResult
praosValidateHeaderSpans ctx ei (maxPV, pvMajor, maxHS, maxBS) tip stateCbor pin arena offs lens
                         verdicts bits = do
  let n = VS.length offs
  when (VS.length lens /= n || VSM.length verdicts /= n || VSM.length bits /= n) $
    throwIO (PraosBatchError (-1) "praosValidateHeaderSpans: vector lengths differ")
  BSU.unsafeUseAsCStringLen arena $ \(ap, alen) ->
    VS.unsafeWith offs $ \offp -> VS.unsafeWith lens $ \lenp ->
    VSM.unsafeWith verdicts $ \verdict -> VSM.unsafeWith bits $ \bitp ->
    allocaBytes 40 $ \hb -> allocaArray n $ \(pidx :: Ptr Int32) ->
    -- decoded fields: slot, block no, ocert n (8 B each), prev hash, cold vk, header hash (32 B
    -- each), body size (4 B), prev-is-genesis (1 B), the nonce value of the certified VRF
    -- output (32 B, the fold evolves the nonce with it) = 157 B per header, one allocation
    allocaBytes (157 * n) $ \decbuf ->
    allocaBytes 168 $ \dec -> allocaBytes 40 $ \out -> allocaBytes 120 $ \hv -> allocaBytes 120 $ \env ->
    alloca $ \stopp -> alloca $ \donep ->
    withChainState stateCbor (n + 65536) $ \st -> withEpochInfo ei $ \eip -> do
      let slot = decbuf :: Ptr Word64
          bno = decbuf `plusPtr` (8 * n) :: Ptr Word64
          ocn = decbuf `plusPtr` (16 * n) :: Ptr Word64
          prev = decbuf `plusPtr` (24 * n) :: Ptr Word8
          cold = decbuf `plusPtr` (56 * n) :: Ptr Word8
          hh = decbuf `plusPtr` (88 * n) :: Ptr Word8
          bsz = decbuf `plusPtr` (120 * n) :: Ptr Word32
          gen = decbuf `plusPtr` (124 * n) :: Ptr Word8
          nonce = decbuf `plusPtr` (125 * n) :: Ptr Word8
      pokeByteOff hb 0 (fromIntegral n :: CSize) >> pokeByteOff hb 8 ap
      pokeByteOff hb 16 (fromIntegral alen :: CSize)
      pokeByteOff hb 24 offp >> pokeByteOff hb 32 lenp
      fillBytes out 0 40 >> pokeByteOff out 0 bitp >> pokeByteOff out 8 pidx >> pokeByteOff out 32 nonce
      fillBytes dec 0 168
      pokeByteOff dec 8 bno >> pokeByteOff dec 16 slot >> pokeByteOff dec 24 prev >> pokeByteOff dec 32 gen
      pokeByteOff dec 40 cold >> pokeByteOff dec 72 bsz >> pokeByteOff dec 96 ocn >> pokeByteOff dec 160 hh
      withRegisteredArena ctx pin (castPtr ap) alen $ verifyHeaderBytes ctx (castPtr hb) (castPtr out) (castPtr dec)
      fillBytes hv 0 120
      pokeByteOff hv 0 (fromIntegral n :: CSize) >> pokeByteOff hv 8 slot >> pokeByteOff hv 16 cold
      pokeByteOff hv 56 ocn
      fillBytes env 0 120
      pokeByteOff env 0 bno >> pokeByteOff env 8 hh >> pokeByteOff env 16 lenp >> pokeByteOff env 24 bsz
      case tip of
        Nothing -> pokeByteOff env 32 (1 :: Int32)
        Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
      pokeByteOff env 88 maxPV >> pokeByteOff env 96 pvMajor >> pokeByteOff env 104 maxHS
      pokeByteOff env 112 maxBS
      checkCtx (ctxPtr ctx) (c_validate_headers (ctxPtr ctx) (castPtr hv) prev gen (castPtr out) (castPtr env) eip st
                                                verdict stopp donep)
      stop <- peek stopp
      st' <- encodeChainState st
      origin :: Int32 <- peekByteOff env 32
      tip' <- if origin /= 0 then pure Nothing else do
        s <- peekByteOff env 40
        b <- peekByteOff env 48
        h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
        pure (Just (s, b, h))
      pure (SpanResult (fromIntegral stop) st' tip')

-- ---------------------------------------------------------------- TPraos headers from stored bytes

-- | tickChainDepState's epoch nonce for TPraos (TICKN: candidate ⭒ lastEpochBlock ⭒ the
-- extra entropy of the protocol parameters; Nothing = NeutralNonce).
praosTickedEpochNonceTPraos :: BS.ByteString -> (Word64, Word64, Word64, Word64) -> Word64 -> Maybe BS.ByteString
                            -> IO (Maybe BS.ByteString)
praosTickedEpochNonceTPraos stateCbor ei slot extra =
  withChainState stateCbor (1 + 65536) $ \st -> withEpochInfo ei $ \eip -> allocaBytes 36 $ \xe ->
  allocaBytes 36 $ \out -> do
    pokeNonce xe 0 extra
    rc <- c_tpraos_ticked_epoch_nonce st eip slot (castPtr xe) (castPtr out)
    when (rc /= 0) $ throwIO (PraosBatchError (fromIntegral rc) "praos_tpraos_ticked_epoch_nonce")
    peekNonce out 0

-- | The decentralisation overlay of a TPraos ledger view (praos_overlay): d = lvD, f =
-- activeSlotVal, the fixed-size epoch layout, and lvGenDelegs as (genesis key hash, delegate
-- cold-key hash, delegate VRF key hash) triples.
data OverlayC = OverlayC
  { ovD           :: !Rational
  , ovF           :: !Rational
  , ovEpochBase   :: !Word64
  , ovEpochLength :: !Word64
  , ovGenDelegs   :: ![(BS.ByteString, BS.ByteString, BS.ByteString)]
  }

-- | praos_set_overlay (every member of a group): Nothing = no overlay (d = 0).
-- struct praos_gen_deleg (88 bytes): genesis_hash28@0 delegate_hash28@28 vrf_hash32@56
-- struct praos_overlay (64 bytes): d_num@0 d_den@8 asc_num@16 asc_den@24 epoch_base_slot@32 epoch_length@40 gen_delegs@48 n_gen_delegs@56
praosSetOverlay :: PraosBatchCtx -> Maybe OverlayC -> IO ()
praosSetOverlay ctx Nothing = check ctx $ case ctx of
  PraosBatchCtx p -> c_set_overlay p nullPtr
  PraosBatchGroup g _ _ -> c_group_set_overlay g nullPtr
praosSetOverlay ctx (Just OverlayC {ovD, ovF, ovEpochBase, ovEpochLength, ovGenDelegs}) =
  allocaBytes (88 * max 1 (length ovGenDelegs)) $ \gd -> allocaBytes 64 $ \ov -> do
    forM_ (zip [0 ..] ovGenDelegs) $ \(i, (gk, dk, vrf)) -> do
      let q = gd `plusPtr` (88 * i)
      pokeBS q 0 gk >> pokeBS q 28 dk >> pokeBS q 56 vrf
    fillBytes ov 0 64
    pokeByteOff ov 0 (fromIntegral (numerator ovD) :: Word64) >> pokeByteOff ov 8 (fromIntegral (denominator ovD) :: Word64)
    pokeByteOff ov 16 (fromIntegral (numerator ovF) :: Word64) >> pokeByteOff ov 24 (fromIntegral (denominator ovF) :: Word64)
    pokeByteOff ov 32 ovEpochBase >> pokeByteOff ov 40 ovEpochLength
    pokeByteOff ov 48 gd >> pokeByteOff ov 56 (fromIntegral (length ovGenDelegs) :: Word32)
    check ctx $ case ctx of
      PraosBatchCtx p -> c_set_overlay p (castPtr ov)
      PraosBatchGroup g _ _ -> c_group_set_overlay g (castPtr ov)

-- | One epoch's stored TPraos headers validated (TPraos.updateChainDepState over the
-- batch, TPraos.hs:378-387, with the envelope): verdicts (PRAOS_V_OK / _ENV_* / _INPUT /
-- PRAOS_V_TPRAOS), the PRTCL predicate-failure set of each header (PRAOS_TPF_*), the chain
-- stop and the state / tip after it.
data TPraosBatchResult = TPraosBatchResult
  { tbrVerdicts  :: ![Word8]
  , tbrFailures  :: ![Word16]
  , tbrBits      :: ![Word16]
  , tbrChainStop :: !Int
  , tbrState     :: !BS.ByteString
  , tbrTip       :: !(Maybe (Word64, Word64, BS.ByteString))
  }

-- | praos_verify_tpraos_header_bytes (BHeader decode + OCERT, KES, both VRF certificates
-- and the 2^512 leader test on the GPU) then praos_tpraos_update_chain_dep_state.  The
-- epoch must have been installed with 'praosSetEpoch' under
-- 'praosTickedEpochNonceTPraos''s nonce.
praosValidateTPraosHeaderBytes :: PraosBatchCtx -> (Word64, Word64, Word64, Word64) -> EnvLimits
                               -> Maybe BS.ByteString -> Maybe (Word64, Word64, BS.ByteString) -> BS.ByteString
                               -> [BS.ByteString] -> IO TPraosBatchResult
praosValidateTPraosHeaderBytes ctx ei (maxPV, pvMajor, maxHS, maxBS) extra tip stateCbor hdrs = do
  let n = length hdrs
      arena = BS.concat hdrs
      lens = map BS.length hdrs
      offs = take n (scanl (+) 0 lens)
  BSU.unsafeUseAsCString arena $ \ap ->
    withArray (map fromIntegral offs :: [Word64]) $ \offp ->
    withArray (map fromIntegral lens :: [Word32]) $ \lenp ->
    allocaBytes 40 $ \hb ->
    allocaArray n $ \(bits :: Ptr Word16) -> allocaArray n $ \(pidx :: Ptr Int32) ->
    allocaBytes (32 * n) $ \nonce ->
    allocaArray n $ \(slot :: Ptr Word64) -> allocaArray n $ \(bno :: Ptr Word64) ->
    allocaArray n $ \(ocn :: Ptr Word64) -> allocaArray n $ \(bsz :: Ptr Word32) ->
    allocaBytes (32 * n) $ \prev -> allocaBytes n $ \gen -> allocaBytes (32 * n) $ \cold ->
    allocaBytes (32 * n) $ \hh -> allocaBytes 168 $ \dec -> allocaBytes 40 $ \out ->
    allocaBytes 136 $ \th -> allocaBytes 120 $ \env -> allocaBytes 36 $ \xe ->
    allocaArray n $ \(verdict :: Ptr Word8) -> allocaArray n $ \(fails :: Ptr Word16) ->
    alloca $ \stopp -> alloca $ \donep ->
    withChainState stateCbor (n + 65536) $ \st -> withEpochInfo ei $ \eip -> do
      pokeByteOff hb 0 (fromIntegral n :: CSize) >> pokeByteOff hb 8 ap
      pokeByteOff hb 16 (fromIntegral (BS.length arena) :: CSize)
      pokeByteOff hb 24 offp >> pokeByteOff hb 32 lenp
      -- praos_tpraos_out: bits, pool_idx, (beta_eta, beta_leader not needed), nonce
      fillBytes out 0 40 >> pokeByteOff out 0 bits >> pokeByteOff out 8 pidx >> pokeByteOff out 32 nonce
      fillBytes dec 0 168
      pokeByteOff dec 8 bno >> pokeByteOff dec 16 slot >> pokeByteOff dec 24 prev >> pokeByteOff dec 32 gen
      pokeByteOff dec 40 cold >> pokeByteOff dec 72 bsz >> pokeByteOff dec 96 ocn >> pokeByteOff dec 160 hh
      verifyTPraosHeaderBytes ctx (castPtr hb) (castPtr out) (castPtr dec)
      -- praos_tpraos_headers: h = praos_headers (n, slot, cold_vk, ocert_n read by the fold)
      fillBytes th 0 136
      pokeByteOff th 0 (fromIntegral n :: CSize) >> pokeByteOff th 8 slot >> pokeByteOff th 16 cold
      pokeByteOff th 56 ocn
      fillBytes env 0 120
      pokeByteOff env 0 bno >> pokeByteOff env 8 hh >> pokeByteOff env 16 lenp >> pokeByteOff env 24 bsz
      case tip of
        Nothing -> pokeByteOff env 32 (1 :: Int32)
        Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
      pokeByteOff env 88 maxPV >> pokeByteOff env 96 pvMajor >> pokeByteOff env 104 maxHS
      pokeByteOff env 112 maxBS
      pokeNonce xe 0 extra
      checkCtx (ctxPtr ctx) (c_tpraos_update_chain_dep_state (ctxPtr ctx) (castPtr th) prev gen (castPtr out)
                                                             (castPtr env) eip (castPtr xe) st verdict fails stopp donep)
      stop <- peek stopp
      vs <- peekArray n verdict
      fs <- peekArray n fails
      bs <- peekArray n bits
      st' <- encodeChainState st
      origin :: Int32 <- peekByteOff env 32
      tip' <- if origin /= 0 then pure Nothing else do
        s <- peekByteOff env 40
        b <- peekByteOff env 48
        h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
        pure (Just (s, b, h))
      pure (TPraosBatchResult vs fs bs (fromIntegral stop) st' tip')

-- | 'praosValidateTPraosHeaderBytes' over Storable vectors (as 'praosValidateHeaderSpans'):
-- verdicts (PRAOS_V_*), PRTCL failure sets (PRAOS_TPF_*) and check bits written into the
-- caller's vectors.  The epoch must have been installed with 'praosSetEpoch' under
-- 'praosTickedEpochNonceTPraos''s nonce.
praosValidateTPraosHeaderSpans :: PraosBatchCtx -> (Word64, Word64, Word64, Word64) -> EnvLimits -> Maybe BS.ByteString
                               -> Maybe (Word64, Word64, BS.ByteString) -> BS.ByteString -> ArenaPin -> BS.ByteString
                               -> VS.Vector Word64 -> VS.Vector Word32 -> VSM.IOVector Word8 -> VSM.IOVector Word16
                               -> VSM.IOVector Word16 -> IO SpanResult
praosValidateTPraosHeaderSpans ctx ei (maxPV, pvMajor, maxHS, maxBS) extra tip stateCbor pin arena offs lens verdicts
                               failures bits = do
  let n = VS.length offs
  when (VS.length lens /= n || VSM.length verdicts /= n || VSM.length failures /= n || VSM.length bits /= n) $
    throwIO (PraosBatchError (-1) "praosValidateTPraosHeaderSpans: vector lengths differ")
  BSU.unsafeUseAsCStringLen arena $ \(ap, alen) ->
    VS.unsafeWith offs $ \offp -> VS.unsafeWith lens $ \lenp ->
    VSM.unsafeWith verdicts $ \verdict -> VSM.unsafeWith failures $ \fails -> VSM.unsafeWith bits $ \bitp ->
    allocaBytes 40 $ \hb -> allocaArray n $ \(pidx :: Ptr Int32) ->
    allocaBytes (157 * n) $ \decbuf ->      -- the decoded fields the fold reads (praosValidateHeaderSpans)
    allocaBytes 168 $ \dec -> allocaBytes 40 $ \out -> allocaBytes 136 $ \th -> allocaBytes 120 $ \env ->
    allocaBytes 36 $ \xe -> alloca $ \stopp -> alloca $ \donep ->
    withChainState stateCbor (n + 65536) $ \st -> withEpochInfo ei $ \eip -> do
      let slot = decbuf :: Ptr Word64
          bno = decbuf `plusPtr` (8 * n) :: Ptr Word64
          ocn = decbuf `plusPtr` (16 * n) :: Ptr Word64
          prev = decbuf `plusPtr` (24 * n) :: Ptr Word8
          cold = decbuf `plusPtr` (56 * n) :: Ptr Word8
          hh = decbuf `plusPtr` (88 * n) :: Ptr Word8
          bsz = decbuf `plusPtr` (120 * n) :: Ptr Word32
          gen = decbuf `plusPtr` (124 * n) :: Ptr Word8
          nonce = decbuf `plusPtr` (125 * n) :: Ptr Word8
      pokeByteOff hb 0 (fromIntegral n :: CSize) >> pokeByteOff hb 8 ap
      pokeByteOff hb 16 (fromIntegral alen :: CSize)
      pokeByteOff hb 24 offp >> pokeByteOff hb 32 lenp
      fillBytes out 0 40 >> pokeByteOff out 0 bitp >> pokeByteOff out 8 pidx >> pokeByteOff out 32 nonce
      fillBytes dec 0 168
      pokeByteOff dec 8 bno >> pokeByteOff dec 16 slot >> pokeByteOff dec 24 prev >> pokeByteOff dec 32 gen
      pokeByteOff dec 40 cold >> pokeByteOff dec 72 bsz >> pokeByteOff dec 96 ocn >> pokeByteOff dec 160 hh
      withRegisteredArena ctx pin (castPtr ap) alen $ verifyTPraosHeaderBytes ctx (castPtr hb) (castPtr out) (castPtr dec)
      fillBytes th 0 136
      pokeByteOff th 0 (fromIntegral n :: CSize) >> pokeByteOff th 8 slot >> pokeByteOff th 16 cold
      pokeByteOff th 56 ocn
      fillBytes env 0 120
      pokeByteOff env 0 bno >> pokeByteOff env 8 hh >> pokeByteOff env 16 lenp >> pokeByteOff env 24 bsz
      case tip of
        Nothing -> pokeByteOff env 32 (1 :: Int32)
        Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
      pokeByteOff env 88 maxPV >> pokeByteOff env 96 pvMajor >> pokeByteOff env 104 maxHS
      pokeByteOff env 112 maxBS
      pokeNonce xe 0 extra
      checkCtx (ctxPtr ctx) (c_tpraos_update_chain_dep_state (ctxPtr ctx) (castPtr th) prev gen (castPtr out)
                                                             (castPtr env) eip (castPtr xe) st verdict fails stopp donep)
      stop <- peek stopp
      st' <- encodeChainState st
      origin :: Int32 <- peekByteOff env 32
      tip' <- if origin /= 0 then pure Nothing else do
        s <- peekByteOff env 40
        b <- peekByteOff env 48
        h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
        pure (Just (s, b, h))
      pure (SpanResult (fromIntegral stop) st' tip')

-- ---------------------------------------------------------------- ImmutableDB replay

data ReplayStats = ReplayStats
  { rsSkipped, rsHeaders, rsValidated, rsStopIndex :: !Word64
  , rsStopVerdict, rsEpochs, rsBatches, rsChunks :: !Word32
  , rsMsIO, rsMsDevice, rsMsFold, rsMsNonce :: !Double
  } deriving Show

-- | praos_replay_immutable: the header-validation pass of db-analyser over an ImmutableDB
-- directory (chunk + secondary index files), from the given state and tip (Nothing =
-- Origin; otherwise a block of the database to resume after).  Returns the statistics,
-- the final PraosState CBOR and tip.  On a group context (praos_group_replay_immutable)
-- consecutive batches go to the members in turn; the nonce chain and the fold stay single,
-- in chain order, so the result is the one-GPU replay's.
praosReplayImmutable :: PraosBatchCtx -> FilePath -> [(BS.ByteString, BS.ByteString, Integer)] -> PraosParamsC
                     -> (Word64, Word64, Word64, Word64) -> EnvLimits -> Maybe (Word64, Word64, BS.ByteString)
                     -> BS.ByteString -> Int
                     -> IO (ReplayStats, BS.ByteString, Maybe (Word64, Word64, BS.ByteString))
praosReplayImmutable ctx dir pools pp ei (maxPV, pvMajor, maxHS, maxBS) tip stateCbor batchMax =
  withCString dir $ \cdir -> withPools pools $ \pp' np -> withParams pp $ \par ->
  withEpochInfo ei $ \eip -> withChainState stateCbor 65536 $ \st ->
  allocaBytes 120 $ \env -> allocaBytes 80 $ \rs -> do
    fillBytes env 0 120
    case tip of
      Nothing -> pokeByteOff env 32 (1 :: Int32)
      Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
    pokeByteOff env 88 maxPV >> pokeByteOff env 96 pvMajor >> pokeByteOff env 104 maxHS
    pokeByteOff env 112 maxBS
    check ctx $ case ctx of
      PraosBatchCtx p -> c_replay_immutable p cdir pp' np par eip (castPtr env) st (fromIntegral batchMax) nullPtr 0
                                            (castPtr rs)
      PraosBatchGroup g _ _ -> c_group_replay_immutable g cdir pp' np par eip (castPtr env) st (fromIntegral batchMax)
                                                        nullPtr 0 (castPtr rs)
    stats <- ReplayStats <$> peekByteOff rs 0 <*> peekByteOff rs 8 <*> peekByteOff rs 16 <*> peekByteOff rs 24
                         <*> peekByteOff rs 32 <*> peekByteOff rs 36 <*> peekByteOff rs 40 <*> peekByteOff rs 44
                         <*> peekByteOff rs 48 <*> peekByteOff rs 56 <*> peekByteOff rs 64 <*> peekByteOff rs 72
    st' <- encodeChainState st
    origin :: Int32 <- peekByteOff env 32
    tip' <- if origin /= 0 then pure Nothing else do
      s <- peekByteOff env 40
      b <- peekByteOff env 48
      h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
      pure (Just (s, b, h))
    pure (stats, st', tip')

-- | praos_replay_immutable_tpraos: the same replay over a TPraos (Shelley..Alonzo)
-- ImmutableDB (TICKN's extra entropy, Nothing = NeutralNonce).  Also returns the PRTCL
-- failure set of every header up to the stop (PRAOS_TPF_*).
praosReplayImmutableTPraos :: PraosBatchCtx -> FilePath -> [(BS.ByteString, BS.ByteString, Integer)] -> PraosParamsC
                           -> (Word64, Word64, Word64, Word64) -> EnvLimits -> Maybe BS.ByteString
                           -> Maybe (Word64, Word64, BS.ByteString) -> BS.ByteString -> Int -> Int
                           -> IO (ReplayStats, [Word8], [Word16], BS.ByteString, Maybe (Word64, Word64, BS.ByteString))
praosReplayImmutableTPraos ctx dir pools pp ei (maxPV, pvMajor, maxHS, maxBS) extra tip stateCbor
                           batchMax cap =
  withCString dir $ \cdir -> withPools pools $ \pp' np -> withParams pp $ \par ->
  withEpochInfo ei $ \eip -> withChainState stateCbor 65536 $ \st ->
  allocaBytes 120 $ \env -> allocaBytes 80 $ \rs -> allocaBytes 36 $ \xe ->
  allocaArray (max 1 cap) $ \(verdicts :: Ptr Word8) -> allocaArray (max 1 cap) $ \(fails :: Ptr Word16) -> do
    fillBytes env 0 120
    case tip of
      Nothing -> pokeByteOff env 32 (1 :: Int32)
      Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
    pokeByteOff env 88 maxPV >> pokeByteOff env 96 pvMajor >> pokeByteOff env 104 maxHS
    pokeByteOff env 112 maxBS
    pokeNonce xe 0 extra
    check ctx $ case ctx of
      PraosBatchCtx p -> c_replay_immutable_tpraos p cdir pp' np par eip (castPtr xe) (castPtr env) st
                                                   (fromIntegral batchMax) verdicts fails (fromIntegral cap) (castPtr rs)
      PraosBatchGroup g _ _ -> c_group_replay_immutable_tpraos g cdir pp' np par eip (castPtr xe) (castPtr env) st
                                                               (fromIntegral batchMax) verdicts fails
                                                               (fromIntegral cap) (castPtr rs)
    stats <- ReplayStats <$> peekByteOff rs 0 <*> peekByteOff rs 8 <*> peekByteOff rs 16 <*> peekByteOff rs 24
                         <*> peekByteOff rs 32 <*> peekByteOff rs 36 <*> peekByteOff rs 40 <*> peekByteOff rs 44
                         <*> peekByteOff rs 48 <*> peekByteOff rs 56 <*> peekByteOff rs 64 <*> peekByteOff rs 72
    let upto = min cap (fromIntegral (rsHeaders stats))
    vs <- peekArray upto verdicts
    fs <- peekArray upto fails
    st' <- encodeChainState st
    origin :: Int32 <- peekByteOff env 32
    tip' <- if origin /= 0 then pure Nothing else do
      s <- peekByteOff env 40
      b <- peekByteOff env 48
      h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
      pure (Just (s, b, h))
    pure (stats, vs, fs, st', tip')

-- | A LedgerView as the ABI takes it (praos_ledger_view): from which epoch on it holds, the
-- PoolDistr entries and the envelope limits (pvMajor lvProtocolVersion, lvMaxHeaderSize,
-- lvMaxBodySize).  db-analyser forecasts one per epoch from the ledger state it advances
-- (Analysis.hs:564-572; all of them change only at an epoch boundary).
data LedgerViewC = LedgerViewC
  { lvcFirstEpoch :: !Word64
  , lvcPools      :: ![(BS.ByteString, BS.ByteString, Integer)]
  , lvcProtMajor  :: !Word64
  , lvcMaxHeader  :: !Word64
  , lvcMaxBody    :: !Word64
  }

-- | praos_[group_]replay_immutable_views: 'praosReplayImmutable' with a ledger view per epoch
-- (the list sorted by first epoch; epoch e uses the last view starting at or before it) instead
-- of one for the whole database.  A batch never spans two views; the fold of each batch uses
-- its view's PoolDistr and envelope limits.
praosReplayImmutableViews :: PraosBatchCtx -> FilePath -> [LedgerViewC] -> PraosParamsC
                          -> (Word64, Word64, Word64, Word64) -> Word64 -> Maybe (Word64, Word64, BS.ByteString)
                          -> BS.ByteString -> Int
                          -> IO (ReplayStats, BS.ByteString, Maybe (Word64, Word64, BS.ByteString))
praosReplayImmutableViews ctx dir views pp ei maxPV tip stateCbor batchMax =
  withCString dir $ \cdir -> withViews views $ \vp nv -> withParams pp $ \par ->
  withEpochInfo ei $ \eip -> withChainState stateCbor 65536 $ \st ->
  allocaBytes 120 $ \env -> allocaBytes 80 $ \rs -> do
    fillBytes env 0 120
    case tip of
      Nothing -> pokeByteOff env 32 (1 :: Int32)
      Just (s, b, h) -> pokeByteOff env 40 s >> pokeByteOff env 48 b >> pokeBS env 56 h
    pokeByteOff env 88 maxPV             -- the limits of each view come from the view
    check ctx $ case ctx of
      PraosBatchCtx p -> c_replay_immutable_views p cdir vp nv par eip (castPtr env) st (fromIntegral batchMax)
                                                  nullPtr 0 (castPtr rs)
      PraosBatchGroup g _ _ -> c_group_replay_immutable_views g cdir vp nv par eip (castPtr env) st
                                                              (fromIntegral batchMax) nullPtr 0 (castPtr rs)
    stats <- ReplayStats <$> peekByteOff rs 0 <*> peekByteOff rs 8 <*> peekByteOff rs 16 <*> peekByteOff rs 24
                         <*> peekByteOff rs 32 <*> peekByteOff rs 36 <*> peekByteOff rs 40 <*> peekByteOff rs 44
                         <*> peekByteOff rs 48 <*> peekByteOff rs 56 <*> peekByteOff rs 64 <*> peekByteOff rs 72
    st' <- encodeChainState st
    origin :: Int32 <- peekByteOff env 32
    tip' <- if origin /= 0 then pure Nothing else do
      s <- peekByteOff env 40
      b <- peekByteOff env 48
      h <- BS.packCStringLen (castPtr (env `plusPtr` 56), 32)
      pure (Just (s, b, h))
    pure (stats, st', tip')

-- | The praos_ledger_view array (48 bytes each), every view's pool array kept alive around it.
withViews :: [LedgerViewC] -> (Ptr () -> Word32 -> IO a) -> IO a
withViews views k = allocaBytes (48 * max 1 (length views)) $ \vp -> go vp (zip [0 ..] views)
  where
    go vp [] = k (castPtr vp) (fromIntegral (length views))
    go vp ((i, LedgerViewC {lvcFirstEpoch, lvcPools, lvcProtMajor, lvcMaxHeader, lvcMaxBody}) : rest) =
      withPools lvcPools $ \pp np -> do
        let q = vp `plusPtr` (48 * i)
        fillBytes q 0 48
        pokeByteOff q 0 lvcFirstEpoch >> pokeByteOff q 8 pp >> pokeByteOff q 16 np
        pokeByteOff q 24 lvcProtMajor >> pokeByteOff q 32 lvcMaxHeader >> pokeByteOff q 40 lvcMaxBody
        go vp rest

-- ---------------------------------------------------------------- ImmutableDB chunk validation

-- | praos_[group_]verify_block_integrity: 'verifyBlockIntegrity' (Shelley/Ledger/Integrity.hs:14-20
-- = verifyHeaderIntegrity, KES at t = max 0 (kp - c0), and blockMatchesHeader, hashTxSeq of the
-- stored segments) of the blocks @arena[off_i .. off_i + len_i)@, in one GPU batch (sharded over
-- a group's members).  Per block 0 (True) or PRAOS_BLK_* bits (1 decode, 2 KES, 4 body hash).
praosVerifyBlockIntegrity :: PraosBatchCtx -> Word64 -> BS.ByteString -> VS.Vector Word64 -> VS.Vector Word32
                          -> IO (VS.Vector Word8)
praosVerifyBlockIntegrity ctx spkp arena offs lens = do
  let n = VS.length offs
  when (VS.length lens /= n) $ throwIO (PraosBatchError (-1) "praosVerifyBlockIntegrity: vector lengths differ")
  res <- VSM.new n
  BSU.unsafeUseAsCStringLen arena $ \(ap, alen) ->
    VS.unsafeWith offs $ \offp -> VS.unsafeWith lens $ \lenp -> VSM.unsafeWith res $ \rp ->
    allocaBytes 40 $ \hb -> do
      pokeByteOff hb 0 (fromIntegral n :: CSize) >> pokeByteOff hb 8 ap
      pokeByteOff hb 16 (fromIntegral alen :: CSize)
      pokeByteOff hb 24 offp >> pokeByteOff hb 32 lenp
      check ctx $ case ctx of
        PraosBatchCtx p -> c_verify_block_integrity p (castPtr hb) spkp rp nullPtr
        PraosBatchGroup g _ _ -> c_group_verify_block_integrity g (castPtr hb) spkp rp nullPtr
  VS.unsafeFreeze res

-- | One chunk's validation outcome: per block Nothing (its CRC matched the secondary index's
-- checksum: trusted without the integrity check) or the PRAOS_BLK_* bits (0 = intact), the first
-- corrupt block and the offset the chunk file is truncated at (its length when none).
data ChunkValidation = ChunkValidation
  { cvResults      :: ![Maybe Word8]
  , cvFirstCorrupt :: !(Maybe Int)
  , cvTruncateAt   :: !Word64
  }

-- | The expensive part of ImmutableDB chunk validation batched on the GPUs: parseChunkFile
-- (ImmutableDB/Impl/Parser.hs:118-141, called from validateChunk, Validation.hs:379-384) runs
-- @checkIntegrity@ (= verifyBlockIntegrity) on every block whose CRC32 does not match the
-- secondary index entry's checksum, in file order, and stops at the first corrupt block,
-- truncating the chunk file at its offset.  Here the blocks are the chunk bytes cut at the
-- entries' block offsets (block i ends where block i+1 starts, the last at the end of the
-- chunk, Secondary.hs:93-128); the CRCs are computed on the host ('computeCRC', as parseChunkFile
-- does for every block anyway) and the mismatching blocks go to 'praosVerifyBlockIntegrity' in
-- one call.  (The block decode, the CRC and the prev-hash line-up stay the reference's; this
-- replaces only the @isNotCorrupt@ calls.  Replayed from C by ffi_harness --chunk.)
verifyChunkIntegrity :: PraosBatchCtx -> Word64 -> (BS.ByteString -> Word32) -> BS.ByteString
                     -> [(Word64, Word32)] -> IO ChunkValidation
verifyChunkIntegrity ctx spkp crc32 chunk entries = do
  let n = length entries
      bounds = zip (map fst entries) (drop 1 (map fst entries) ++ [fromIntegral (BS.length chunk)])
      spans = [ (i, o, e - o) | (i, ((o, e), (_, want))) <- zip [0 ..] (zip bounds entries)
                              , crc32 (BS.take (fromIntegral (e - o)) (BS.drop (fromIntegral o) chunk)) /= want ]
  when (or [ e < o || e > fromIntegral (BS.length chunk) | (o, e) <- bounds ]) $
    throwIO (PraosBatchError (-2) "verifyChunkIntegrity: a secondary index entry outside its chunk")
  res <- praosVerifyBlockIntegrity ctx spkp chunk (VS.fromList [ o | (_, o, _) <- spans ])
                                   (VS.fromList [ fromIntegral l | (_, _, l) <- spans ])
  let checked = zip [ i | (i, _, _) <- spans ] (VS.toList res)
      results = [ lookup i checked | i <- [0 .. n - 1] ]
      firstBad = case [ i | (i, r) <- checked, r /= 0 ] of
        (i : _) -> Just i
        []      -> Nothing
  pure ChunkValidation
    { cvResults = results
    , cvFirstCorrupt = firstBad
    , cvTruncateAt = maybe (fromIntegral (BS.length chunk)) (\i -> fst (entries !! i)) firstBad }

-- ---------------------------------------------------------------- errors

-- | The reference error a verdict stands for, by name (logs, traces).  The typed
-- constructors with their exact payloads (PraosValidationErr, PraosEnvelopeError,
-- HeaderEnvelopeError, the TPraos PRTCL failures) are built by
-- "Ouroboros.Consensus.Protocol.Praos.Batch.Errors".
-- The bits split KES failures into "Reject" (Merkle path, 0x08) and the Ed25519 leaf
-- ("Verification failed", 0x10), as verifySignedKES reports them.
verdictToError :: Word8 -> Word16 -> Maybe String
verdictToError v bits = case v of
  0  -> Nothing
  1  -> Just "KESBeforeStartOCERT"
  2  -> Just "KESAfterEndOCERT"
  3  -> Just "InvalidSignatureOCERT"
  4  -> Just ("InvalidKesSignatureOCERT " ++ if bits .&. 0x08 /= 0 then "Reject" else "Verification failed")
  5  -> Just "NoCounterForKeyHashOCERT"
  6  -> Just "CounterTooSmallOCERT"
  7  -> Just "CounterOverIncrementedOCERT"
  8  -> Just "VRFKeyUnknown"
  9  -> Just "VRFKeyWrongVRFKey"
  10 -> Just "VRFKeyBadProof"
  11 -> Just "VRFLeaderValueTooBig"
  12 -> Just "(undecodable header)"
  13 -> Just "UnexpectedBlockNo"
  14 -> Just "UnexpectedSlotNo"
  15 -> Just "UnexpectedPrevHash"
  16 -> Just "ObsoleteNode"
  17 -> Just "HeaderSizeTooLarge"
  18 -> Just "BlockSizeTooLarge"
  19 -> Just "ChainTransitionError (TPraos PRTCL failures)"
  _  -> Just ("unknown verdict " ++ show v)
