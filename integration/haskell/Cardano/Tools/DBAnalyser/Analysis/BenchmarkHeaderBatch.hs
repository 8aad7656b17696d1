{-# LANGUAGE BangPatterns        #-}
{-# LANGUAGE RankNTypes          #-}
{-# LANGUAGE NamedFieldPuns      #-}
{-# LANGUAGE ScopedTypeVariables #-}

-- | A db-analyser analysis beside 'BenchmarkLedgerOps' (Analysis.hs:75-88, :479-607):
-- header revalidation of a Praos (Babbage/Conway) ImmutableDB in per-epoch batches on the
-- GPUs of one node through 'Ouroboros.Consensus.Protocol.Praos.Batch' (Storable vectors in and
-- out), timed per epoch on the monotonic wall clock, one line per epoch:
--
--   epoch  headers  validated  stop_verdict  ms  headers/s
--
-- A maintainer wires it in as one more 'AnalysisName' constructor
-- (@BenchmarkHeaderBatch (Maybe FilePath) [Int]@: output file, devices) and one more
-- equation of runAnalysis (Analysis.hs:108-123).  The stream is the same
-- 'processAllImmutableDB' loop (Analysis.hs:815-847) with 'GetRawHeader' as the block
-- component, so the bytes the GPU decodes are exactly the stored header spans the
-- secondary index gives (Secondary.hs:93-128).  With several devices each epoch's batch is
-- sharded over them by contiguous slot range (praos_group, SURVEY sec. 8e) and folded once.
--
-- The epoch's headers are appended as they stream into one growing pinned arena with its
-- offset / length vectors (no list of n ByteStrings per epoch: an epoch is 432k headers), and
-- that arena is handed to the batch as it is.  Shipped as source (no GHC here); the ABI
-- calls it makes are replayed from C by integration/c/ffi_harness.c (phases "typed" and
-- "typed_group").
module Cardano.Tools.DBAnalyser.Analysis.BenchmarkHeaderBatch
  ( benchmarkHeaderBatch
  , EpochBatchEnv (..)
  ) where

import           Control.Monad (unless, when)
import qualified Data.ByteString as BS
import qualified Data.ByteString.Internal as BSI
import qualified Data.ByteString.Lazy as BSL
import qualified Data.ByteString.Unsafe as BSU
import           Data.IORef
import qualified Data.Vector.Storable as VS
import qualified Data.Vector.Storable.Mutable as VSM
import           Data.Word (Word16, Word32, Word64, Word8)
import           Foreign.Marshal.Utils (copyBytes)
import           Foreign.Ptr (castPtr, plusPtr)
import           GHC.Clock (getMonotonicTimeNSec)
import qualified System.IO as IO
import           Text.Printf (hPrintf)

import           Ouroboros.Consensus.Protocol.Praos.Batch

-- | What the analysis needs besides the stream: the epoch layout and stability window
-- (praosParams / EpochInfo), the ledger view (PoolDistr, envelope limits) installed per
-- epoch, the protocol parameters, the genesis PraosState (CBOR) and the GPUs to use.
data EpochBatchEnv = EpochBatchEnv
  { ebEpochInfo   :: (Word64, Word64, Word64, Word64)   -- base slot, base epoch, length, window
  , ebEnvLimits   :: (Word64, Word64, Word64, Word64)   -- maxMajorPV, pvMajor, maxHeaderSize, maxBodySize
  , ebPools       :: Word64 -> [(BS.ByteString, BS.ByteString, Integer)]   -- PoolDistr of an epoch
  , ebParams      :: PraosParamsC
  , ebStateCbor   :: BS.ByteString
  , ebDevices     :: [Int]                              -- one device, or a group (8 on one node)
  }

-- | One epoch's headers as they stream in: the header bytes back to back in a growing
-- Storable arena, and each header's offset and length.
data EpochArena = EpochArena
  { eaBytes :: !(VSM.IOVector Word8)
  , eaOffs  :: !(VSM.IOVector Word64)
  , eaLens  :: !(VSM.IOVector Word32)
  , eaLen   :: !Int              -- bytes used
  , eaN     :: !Int              -- headers
  , eaFirst :: !Word64           -- slot of the first header
  }

newArena :: IO EpochArena
newArena = EpochArena <$> VSM.new (64 * 1024 * 1024) <*> VSM.new 65536 <*> VSM.new 65536 <*> pure 0 <*> pure 0 <*> pure 0

-- | Append one stored header (amortised doubling, one copy of its bytes).
pushHeader :: EpochArena -> Word64 -> BS.ByteString -> IO EpochArena
pushHeader a slot raw = do
  let l = BS.length raw
      grow v need = if VSM.length v >= need then pure v else VSM.grow v (max need (VSM.length v))
  bytes <- grow (eaBytes a) (eaLen a + l)
  offs <- grow (eaOffs a) (eaN a + 1)
  lens <- grow (eaLens a) (eaN a + 1)
  VSM.unsafeWith bytes $ \dst -> BSU.unsafeUseAsCString raw $ \src ->
    copyBytes (dst `plusPtr` eaLen a) (castPtr src) l
  VSM.unsafeWrite offs (eaN a) (fromIntegral (eaLen a))
  VSM.unsafeWrite lens (eaN a) (fromIntegral l)
  pure a { eaBytes = bytes, eaOffs = offs, eaLens = lens, eaLen = eaLen a + l, eaN = eaN a + 1
         , eaFirst = if eaN a == 0 then slot else eaFirst a }

-- | @benchmarkHeaderBatch out env stream@: @stream@ is the analysis' processAll over the
-- ImmutableDB with 'GetRawHeader' (slot and raw header bytes per block), folded here into
-- per-epoch batches.
benchmarkHeaderBatch
  :: Maybe FilePath
  -> EpochBatchEnv
  -> (forall st. st -> (st -> (Word64, BSL.ByteString) -> IO (Bool, st)) -> IO st)
  -> IO ()
benchmarkHeaderBatch mOut EpochBatchEnv {ebEpochInfo, ebEnvLimits, ebPools, ebParams, ebStateCbor, ebDevices}
                     stream =
  withOut mOut $ \h -> withPraosBatchDevices ebDevices $ \ctx -> do
    IO.hPutStrLn h ("# devices " ++ show ebDevices ++ " (" ++ show (praosBatchMembers ctx) ++ " contexts)")
    IO.hPutStrLn h "epoch\theaders\tvalidated\tstop_verdict\tms\theaders/s"
    stRef <- newIORef ebStateCbor
    tipRef <- newIORef Nothing
    arena0 <- newArena
    let (base, baseNo, len, _) = ebEpochInfo
        epochOf s = baseNo + (s - base) `div` len
        -- one epoch's batch: tick, install the ledger view, validate, report
        flush e a
          | eaN a == 0 = pure True
          | otherwise = do
              st <- readIORef stRef
              tip <- readIORef tipRef
              let n = eaN a
              offs <- VS.freeze (VSM.slice 0 n (eaOffs a))
              lens <- VS.freeze (VSM.slice 0 n (eaLens a))
              -- the arena as a ByteString over the same pinned buffer (no copy)
              let (fp, _) = VSM.unsafeToForeignPtr0 (eaBytes a)
                  arena = BSI.fromForeignPtr fp 0 (eaLen a)
              eta <- praosTickedEpochNonce st ebEpochInfo (eaFirst a)
              praosSetEpoch ctx eta (ebPools e) ebParams
              verdicts <- VSM.new n :: IO (VSM.IOVector Word8)
              bits <- VSM.new n :: IO (VSM.IOVector Word16)
              -- wall clock around the batch (the foreign call is safe: mutator time would not
              -- count the time the GPUs spend)
              t0 <- getMonotonicTimeNSec
              !r <- praosValidateHeaderSpans ctx ebEpochInfo ebEnvLimits tip st arena offs lens verdicts bits
              t1 <- getMonotonicTimeNSec
              let ms = fromIntegral (t1 - t0) / 1e6 :: Double
                  stopped = srChainStop r < n
              verdict <- if stopped then VSM.read verdicts (srChainStop r) else pure 0
              hPrintf h "%d\t%d\t%d\t%d\t%.3f\t%.0f\n" e n (srChainStop r) verdict ms
                      (fromIntegral n / max 1e-9 (ms / 1e3))
              writeIORef stRef (srState r)
              writeIORef tipRef (srTip r)
              pure (not stopped)          -- the reference stops at the first invalid header
        reset a = a { eaLen = 0, eaN = 0 }
    (e, acc, ok) <- stream (0, arena0, True) $ \(e, acc, ok) (slot, raw) -> do
      let e' = epochOf slot
          hdr = BSL.toStrict raw
      if eaN acc == 0 || e' == e
        then do
          acc' <- pushHeader acc slot hdr
          pure (True, (e', acc', ok))
        else do
          ok' <- flush e acc
          acc' <- pushHeader (reset acc) slot hdr      -- the arena is reused epoch after epoch
          pure (ok', (e', acc', ok'))
    when ok $ do
      _ <- flush e acc
      pure ()
    unless ok $ IO.hPutStrLn h "# stopped at the first invalid header"
  where
    withOut (Just f) k = IO.withFile f IO.WriteMode k
    withOut Nothing k = k IO.stdout
